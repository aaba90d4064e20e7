#!/bin/bash
# L2 hit rate per kernel of one bench render: one rocprofv3 pass of
# TCC_HIT_sum / TCC_MISS_sum (then: python tools/l2_to_profile.py <tag>).
# usage: tools/gpu_l2.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
d=gpurun_out/l2_$tag; mkdir -p $d
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $d -o run -- \
    python3 bench.py --roofline-only "$@" > $d/bench.log 2>&1
rc=$?; echo "l2 $tag rc=$rc"; exit $rc
