#!/bin/bash
# GPU test suite after the discrete-vertex NEE change (D10), interleaved A/B
# against the full NEE (NORI_DISCRETE_NEE=1) at 64 and 512 spp, then the
# finisher profile.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
r=$?; echo "pytest rc=$r"; tail -2 gpurun_out/pytest_gpu.log; [ $r -ne 0 ] && exit $r
for spp in 64 512; do for e in NORI_X=0 NORI_DISCRETE_NEE=1 NORI_X=0 NORI_DISCRETE_NEE=1; do
  env $e timeout -k 10 300 python bench.py --spp $spp --no-cpu-baseline --no-parity > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$e rc=$r"; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spp $e', round(d['value'],1), round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
done; done
NORI_DEBUG=1 NORI_GPU_LIB=$PWD/$L/var/proffin.so timeout -k 10 300 python bench.py --spp 64 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/pf.log 2>&1
r=$?; echo "proffin rc=$r"; grep "finisher" gpurun_out/pf.log | tail -3
exit $r
