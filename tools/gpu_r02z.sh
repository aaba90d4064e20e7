#!/bin/bash
# Termination lookahead once the work streams run dry (NORI_LOOKAHEAD_END,
# default 2; 6 = the old constant lookahead): A/B at the 64-spp share and C2.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1
r=$?; echo "pytest rc=$r"; tail -1 gpurun_out/pytest_parity.log; [ $r -ne 0 ] && exit $r
B="python bench.py --no-cpu-baseline --no-parity --no-roofline"
ab() { t=$1; shift
  env $E timeout -k 10 300 $B "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t [$E]', round(d['value'],1), round(d['ms_per_step'],3))"
}
for rep in 1 2 3; do
  for E in "NORI_LOOKAHEAD_END=6" "NORI_X=0" "NORI_LOOKAHEAD_END=1" "NORI_LOOKAHEAD=3"; do ab s64 --spp 64 --steps 10; done
done
for rep in 1 2; do
  for E in "NORI_LOOKAHEAD_END=6" "NORI_X=0" "NORI_LOOKAHEAD_END=1"; do ab c2; ab s128 --spp 128 --steps 10; done
done
E="NORI_X=0"; ab c5 --config c5 --steps 3 --warmup 1
E="NORI_LOOKAHEAD_END=6"; ab c5 --config c5 --steps 3 --warmup 1
