#!/bin/bash
# One gpurun call: the GPU test suite, smoke(), then bench lines.
#   tools/gpu_suite.sh [--tests 'pytest args'] [--no-tests] [--configs 'c2 c3 ...'] [--s64] [--tag name]
# Logs go to gpurun_out/<tag>/ ; every GPU step has its own time limit and the
# script stops at the first failure (no retries).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tests="tests -m gpu"; run_tests=1; configs="c2"; s64=0; tag=suite
while [ $# -gt 0 ]; do
  case $1 in
    --tests) tests=$2; shift 2;;
    --no-tests) run_tests=0; shift;;
    --configs) configs=$2; shift 2;;
    --s64) s64=1; shift;;
    --tag) tag=$2; shift 2;;
    *) echo "unknown arg $1"; exit 2;;
  esac
done
out=gpurun_out/$tag; mkdir -p $out
if [ $run_tests = 1 ]; then
  timeout -k 10 900 python -u -m pytest $tests -v -rA -s --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1
  r=$?; echo "pytest rc=$r"; grep -E "passed|failed" $out/pytest_gpu.log | tail -1
  if [ $r -ne 0 ]; then grep -E "^FAILED|Error" $out/pytest_gpu.log | head -10; exit $r; fi
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; tail -5 $out/smoke.log; exit 1; }
  grep smoke: $out/smoke.log
fi
for c in $configs; do
  [ $c = none ] && continue
  extra=""; [ $c != c2 ] && extra="--steps 3 --warmup 1"
  timeout -k 10 400 python bench.py --config $c $extra > $out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $out/bench_$c.log; exit 1; }
  grep '^{' $out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value'],1), 'frac', round(d['roofline']['frac'],4), 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value'],2), 'parity', d.get('parity',{}).get('l2'))"
done
if [ $s64 = 1 ]; then
  timeout -k 10 300 python bench.py --spp 64 --steps 10 --no-cpu-baseline --no-parity --no-roofline > $out/bench_s64.log 2>&1 || exit 1
  grep '^{' $out/bench_s64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('s64', round(d['value'],1), round(d['ms_per_step'],3), 'ms')"
fi
exit 0
