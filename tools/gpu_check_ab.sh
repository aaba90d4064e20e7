#!/bin/bash
# One gpurun call: the extension-kernel equivalence tests, then an interleaved
# A/B of bench.py over the given configurations (tools/gpu_ab.sh syntax;
# "@name" stands for NORI_GPU_LIB=<repo>/nori-ray-tracer_amd/lib/libnori_gpu_name.so).
# usage: REPS=2 tools/gpu_check_ab.sh "cfg1 cfg2 ..." [bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_results.txt
cfgs=""
for c in $1; do
  case $c in @*) c="NORI_GPU_LIB=$GRAFT_REPO_ROOT/nori-ray-tracer_amd/lib/libnori_gpu_${c#@}.so";; esac
  cfgs="$cfgs $c"
done
shift
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_extend_bin.py} \
      > gpurun_out/check.log 2>&1
  r=$?; grep -E "passed|failed|skipped|PASS|FAIL" gpurun_out/check.log | tail -12
  [ $r -eq 0 ] || exit $r
fi
bash tools/gpu_ab.sh "$cfgs" "$@"
