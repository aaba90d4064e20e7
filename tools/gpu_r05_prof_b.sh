#!/bin/bash
# Round-5 profiles, part B: C4 and C5.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for c in c4 c5; do bash tools/gpu_profile_all.sh r05_$c --config $c --roofline-only || exit $?; done
exit 0
