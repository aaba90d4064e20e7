#!/bin/bash
# Bench of the current library (twice), then the finisher profile build at 64 and 512 spp.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/ab_main_$rep.log 2>&1
  r=$?; echo "main rc=$r"; [ $r -ne 0 ] && exit $r
  grep '^{' gpurun_out/ab_main_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(' ', round(d['value'],1), {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
done
for spp in 64 512; do
  NORI_DEBUG=1 NORI_GPU_LIB=$PWD/$L/var/proffin.so timeout -k 10 300 python bench.py --spp $spp --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/pf_$spp.log 2>&1
  r=$?; echo "proffin $spp rc=$r"; [ $r -ne 0 ] && exit $r
  grep "finisher" gpurun_out/pf_$spp.log | tail -3
done
exit 0
