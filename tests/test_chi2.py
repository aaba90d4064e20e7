"""The reference's chi^2 test of BSDF sampling (SURVEY.md 8c fixture 5):
scenes/pa3/tests/chi2test-microfacet.xml, three microfacet configurations,
ChiSquareTest defaults (chi2test.cpp:44-73): 10 cos(theta) x 20 phi cells,
1M samples and 5 incident directions per BSDF, minExpFrequency 5, alpha 0.01
Sidak-corrected over the 15 tests.  The oracle's Microfacet::sample is binned
(chi2test.cpp:124-142) and Microfacet::pdf is integrated over every cell
(chi2test.cpp:147-175; Gauss-Legendre 24 x 24 per cell here instead of the
reference's adaptive Simpson, hypothesis.h:61-101), then hypothesis::chi2_test
(ext/hypothesis/hypothesis.h:140-230) is restated below.  No GPU needed.
"""
import xml.etree.ElementTree as ET

import numpy as np
from scipy import special, stats

import nori_amd
import pyoracle
from conftest import scene_path


def chi2_test(obs, exp, sample_count, min_exp, alpha, num_tests):
    """hypothesis::chi2_test (hypothesis.h:140-230): pool cells of low expected
    frequency (in increasing order), chi^2 statistic, p-value, Sidak level."""
    order = np.argsort(exp, kind="stable")
    pooled_f = pooled_e = chsq = 0.0
    dof = 0
    for i in order:
        if exp[i] == 0:
            if obs[i] > sample_count * 1e-5:
                return False, "samples in a cell of expected frequency 0"
        elif exp[i] < min_exp or (0 < pooled_e < min_exp):
            pooled_f += obs[i]
            pooled_e += exp[i]
        else:
            chsq += (obs[i] - exp[i]) ** 2 / exp[i]
            dof += 1
    if pooled_e > 0 or pooled_f > 0:
        chsq += (pooled_f - pooled_e) ** 2 / pooled_e
        dof += 1
    dof -= 1
    if dof <= 0:
        return False, f"too few degrees of freedom ({dof})"
    pval = 1.0 - stats.chi2.cdf(chsq, dof)
    level = 1.0 - (1.0 - alpha) ** (1.0 / num_tests)
    return bool(pval >= level), f"chi^2 = {chsq:.1f}, dof = {dof}, p = {pval:.4f}, level = {level:.5f}"


def _bsdfs():
    root = ET.parse(scene_path("pa3", "tests", "chi2test-microfacet.xml")).getroot()
    out = []
    for b in root.iter("bsdf"):
        d = nori_amd._abi.BsdfDesc()
        d.type = nori_amd._abi.BSDF_MICROFACET
        props = {p.get("name"): p.get("value") for p in b}
        d.alpha = float(props["alpha"])
        d.int_ior = float(props["intIOR"])
        d.ext_ior = float(props["extIOR"])
        d.kd[:] = [float(x) for x in props["kd"].replace(",", " ").split()]
        out.append(d)
    return out


def test_microfacet_chi2(built):
    res_t, res_p, n, tests_per_bsdf = 10, 20, 10 * 20 * 5000, 5
    bsdfs = _bsdfs()
    assert len(bsdfs) == 3
    rng = np.random.default_rng(2024)
    gx, gw = special.roots_legendre(24)
    fails = []
    for b in bsdfs:
        for _ in range(tests_per_bsdf):
            ct = rng.random()
            st, ph = np.sqrt(max(0.0, 1 - ct * ct)), 2 * np.pi * rng.random()
            wi = np.array([np.cos(ph) * st, np.sin(ph) * st, ct], np.float32)
            # chi2test.cpp:124-142: bin the sampled directions (zero-weight samples skipped)
            smp = pyoracle.bsdf_sample(b, np.tile(wi, (n, 1)), rng.random((n, 2), dtype=np.float32))
            keep = smp[:, 3] != 0
            wo = smp[keep, :3]
            tb = np.clip(np.floor((wo[:, 2] * 0.5 + 0.5) * res_t).astype(int), 0, res_t - 1)
            sp = np.arctan2(wo[:, 1], wo[:, 0]) * (1 / (2 * np.pi))
            sp = np.where(sp < 0, sp + 1, sp)
            pb = np.clip(np.floor(sp * res_p).astype(int), 0, res_p - 1)
            obs = np.bincount(tb * res_p + pb, minlength=res_t * res_p).astype(np.float64)
            # chi2test.cpp:147-175: integrate pdf over each (cos theta, phi) cell
            exp = np.zeros(res_t * res_p)
            for i in range(res_t):
                c0, c1 = -1 + i * 2 / res_t, -1 + (i + 1) * 2 / res_t
                cs = 0.5 * (c1 - c0) * gx + 0.5 * (c1 + c0)
                for j in range(res_p):
                    p0, p1 = j * 2 * np.pi / res_p, (j + 1) * 2 * np.pi / res_p
                    phs = 0.5 * (p1 - p0) * gx + 0.5 * (p1 + p0)
                    C, P = np.meshgrid(cs, phs, indexing="ij")
                    S = np.sqrt(1 - C * C)
                    wo_q = np.stack([S * np.cos(P), S * np.sin(P), C], -1).reshape(-1, 3).astype(np.float32)
                    pdf = pyoracle.bsdf_eval_pdf(b, np.tile(wi, (wo_q.shape[0], 1)), wo_q)[:, 3].reshape(C.shape)
                    w2 = np.outer(gw, gw) * 0.25 * (c1 - c0) * (p1 - p0)
                    exp[i * res_p + j] = float((pdf * w2).sum()) * n
            ok, msg = chi2_test(obs, exp, n, 5, 0.01, tests_per_bsdf * len(bsdfs))
            print(f"alpha {b.alpha}: {msg}")
            if not ok:
                fails.append((b.alpha, msg))
    assert not fails, fails
