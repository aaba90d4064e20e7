#!/bin/bash
# Finisher phase clocks (NORI_PROF_FINISH build) at 64 and 512 spp.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
for spp in 64 512; do
  NORI_DEBUG=1 NORI_GPU_LIB=$PWD/$L/var/proffin.so timeout -k 10 300 python bench.py --spp $spp --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/pf_$spp.log 2>&1
  r=$?; echo "proffin $spp rc=$r"; [ $r -ne 0 ] && exit $r
  grep "finisher\|chunk" gpurun_out/pf_$spp.log | tail -3
done
exit 0
