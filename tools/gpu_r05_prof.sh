#!/bin/bash
# Round-5 evidence, part 2: rocprofv3 kernel traces, HBM (FETCH/WRITE) and SQ
# counter passes of the roofline render for C2-C5, and the C3 L2 hit rates.
# Then on the CPU: python tools/pmc_to_profile.py r05[_c3|_c4|_c5]; python tools/l2_to_profile.py r05_c3
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_profile_all.sh r05 --roofline-only || exit $?
for c in c3 c4 c5; do bash tools/gpu_profile_all.sh r05_$c --config $c --roofline-only || exit $?; done
bash tools/gpu_l2.sh r05_c3 --config c3 || exit $?
exit 0
