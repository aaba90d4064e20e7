#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (writes gpurun_out/prof_<tag>/).
# usage: tools/gpu_prof.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/prof_$tag
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
    python3 bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/prof_$tag/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_$tag -type f | head -20; exit $rc
