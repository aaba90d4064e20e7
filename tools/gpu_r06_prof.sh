#!/bin/bash
# Round-6 profiles in one GPU call: for C2-C5, the kernel trace + stats, the
# HBM counters (FETCH_SIZE / WRITE_SIZE, one pass each) and two SQ passes of
# the render bench.py times its roofline on (--roofline-only: one pool part,
# kernels serialised); the C3 L2 pass.  Then, on the CPU:
#   for t in r06 r06_c3 r06_c4 r06_c5; do python tools/pmc_to_profile.py $t; done
#   python tools/l2_to_profile.py r06_c3
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_profile_all.sh r06 --roofline-only || exit $?
for c in c3 c4 c5; do bash tools/gpu_profile_all.sh r06_$c --config $c --roofline-only || exit $?; done
bash tools/gpu_l2.sh r06_c3 --config c3 || exit $?
exit 0
