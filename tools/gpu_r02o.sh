#!/bin/bash
# Work-queue splat (narrow beside the finisher + wide after it) vs the fixed
# grid (NORI_SPLAT_PASSES set = the round-1 grid): parity, then C2/C4/C5/64spp.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_outputs.py tests/test_gpu_torch.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_par.log 2>&1
r=$?; echo "parity rc=$r"; tail -1 gpurun_out/pytest_par.log; [ $r -ne 0 ] && exit $r
ab() { # tag env args...
  t=$1; e=$2; shift 2
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $e rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $e', round(d['value'],1), round(d['ms_per_step'],2))"
}
for rep in 1 2; do
  ab c2 NORI_X=0; ab c2 NORI_SPLAT_PASSES=512
  ab s64 NORI_X=0 --spp 64; ab s64 NORI_SPLAT_PASSES=64 --spp 64
  ab c4 NORI_X=0 --config c4 --steps 3 --warmup 1; ab c4 NORI_SPLAT_PASSES=1024 --config c4 --steps 3 --warmup 1
  ab c5 NORI_X=0 --config c5 --steps 3 --warmup 1; ab c5 NORI_SPLAT_PASSES=2048 --config c5 --steps 3 --warmup 1
done
