#!/bin/bash
# SQ_INSTS_VALU / SQ_WAVES per kernel for every library under lib/var (and the default one).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for lib in nori-ray-tracer_amd/lib/libnori_gpu.so nori-ray-tracer_amd/lib/var/*.so; do
  n=$(basename $lib .so)
  d=gpurun_out/pmcv_$n
  mkdir -p $d
  NORI_GPU_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $d -o run -- \
     python3 bench.py --steps 1 --warmup 0 --no-parity --no-cpu-baseline > $d/bench.log 2>&1
  rc=$?; echo "$n rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
