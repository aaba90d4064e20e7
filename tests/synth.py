"""Deterministic synthetic scenes for the tests: the generators live with the
BASELINE configurations in nori_amd.configs (bench.py builds C3/C4 from them)."""
from nori_amd.configs import CBOX, DISNEY, cbox_variant, envmap_image, envmap_scene, heightfield_obj, heightfield_scene  # noqa: F401
