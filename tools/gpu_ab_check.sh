#!/bin/bash
# One gpurun call: the trace-equivalence and parity tests, then an interleaved
# A/B of bench.py (tools/gpu_ab.sh syntax; "@name" = NORI_GPU_LIB=<lib>/libnori_gpu_name.so).
# usage: REPS=3 tools/gpu_ab_check.sh "cfg1 cfg2 ..." [bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
cfgs=$1
shift
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $PT tests/test_gpu_pair_filter.py tests/test_gpu_parity.py -k "not multirank" > gpurun_out/abcheck.log 2>&1
r=$?; echo "tests rc=$r: $(tail -1 gpurun_out/abcheck.log)"; [ $r -eq 0 ] || exit $r
rm -f gpurun_out/ab_results.txt
bash tools/gpu_ab.sh "$cfgs" "$@"
