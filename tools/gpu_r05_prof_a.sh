#!/bin/bash
# Round-5 profiles, part A: C2 and C3 (kernel trace, FETCH/WRITE, SQ passes) and the C3 L2 pass.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_profile_all.sh r05 --roofline-only || exit $?
bash tools/gpu_profile_all.sh r05_c3 --config c3 --roofline-only || exit $?
bash tools/gpu_l2.sh r05_c3 --config c3 || exit $?
exit 0
