#!/bin/bash
# 52-byte path state (prev/invz, work/flag and the pcg32 state folded into
# the ray and throughput words, the stream increment recomputed): full GPU
# suite, then A/B against the previous layout on C2 (512 / 64 spp), C4, C5.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
r=$?; echo "pytest rc=$r"; tail -1 gpurun_out/pytest_gpu.log; [ $r -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -5; exit $r; }
ab() { t=$1; v=$2; shift 2
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v', round(d['value'],1), round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
}
for rep in 1 2; do
  for v in libnori_gpu var/old; do ab c2 $v; done
  for v in libnori_gpu var/old; do ab s64 $v --spp 64; done
done
for v in libnori_gpu var/old; do ab c4 $v --config c4 --steps 3 --warmup 1; ab c5 $v --config c5 --steps 3 --warmup 1; done
