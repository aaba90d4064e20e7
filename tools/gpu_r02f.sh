#!/bin/bash
# Parity after the cooperative-scan change, A/B of the coop threshold at 64 and
# 512 spp, then finisher profiles with and without NEE work.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_par.log 2>&1
r=$?; echo "parity rc=$r"; tail -2 gpurun_out/pytest_par.log; [ $r -ne 0 ] && exit $r
for spp in 64 512; do for v in libnori_gpu var/coop8 libnori_gpu var/coop8; do
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --spp $spp --no-cpu-baseline --no-parity > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$v rc=$r"; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spp $v', round(d['value'],1), round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
done; done
for v in proffin proffin_nonee; do
  NORI_DEBUG=1 NORI_GPU_LIB=$PWD/$L/var/$v.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/pf_$v.log 2>&1
  r=$?; echo "$v rc=$r"; [ $r -ne 0 ] && exit $r
  grep "finisher" gpurun_out/pf_$v.log | tail -3
done
exit 0
