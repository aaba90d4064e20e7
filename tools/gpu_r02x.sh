#!/bin/bash
# Tail finisher spread over ~2048 waves (K = n/2048 paths per wave) against
# 64 paths per wave (fw0) and ~8192 waves (fw8k): parity, then A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
r=$?; echo "pytest rc=$r"; tail -1 gpurun_out/pytest_gpu.log; [ $r -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -5; exit $r; }
ab() { t=$1; v=$2; shift 2
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --no-roofline "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v', round(d['value'],1), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  for v in libnori_gpu var/fw0 var/fw8k; do ab s64 $v --spp 64 --steps 10; done
done
for v in libnori_gpu var/fw0 var/fw8k; do ab c2 $v; done
for v in libnori_gpu var/fw0; do ab c5 $v --config c5 --steps 3 --warmup 1; ab c4 $v --config c4 --steps 3 --warmup 1; done
for v in libnori_gpu var/fw0; do ab c3 $v --config c3 --steps 3 --warmup 1; done
