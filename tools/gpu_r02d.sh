#!/bin/bash
# A/B of the shadow record update and 2 rays per thread in the scan kernels,
# then the finisher's longest-wave span (NORI_PROF_FINISH build) at 64 and 512 spp.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
for rep in 1 2; do
for v in libnori_gpu var/k2; do
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/ab_$(basename $v)_$rep.log 2>&1
  r=$?; echo "$v rc=$r"; [ $r -ne 0 ] && exit $r
  grep '^{' gpurun_out/ab_$(basename $v)_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(' ', round(d['value'],1), {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
done; done
for spp in 64 512; do
  NORI_DEBUG=1 NORI_GPU_LIB=$PWD/$L/var/proffin.so timeout -k 10 300 python bench.py --spp $spp --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/pf_$spp.log 2>&1
  r=$?; echo "proffin $spp rc=$r"; [ $r -ne 0 ] && exit $r
  grep "finisher" gpurun_out/pf_$spp.log | tail -2
done
exit 0
