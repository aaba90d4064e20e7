#!/bin/bash
# Bench each library variant under nori-ray-tracer_amd/lib/var (tuning sweeps).
# usage: tools/gpu_variants.sh [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in nori-ray-tracer_amd/lib/libnori_gpu.so nori-ray-tracer_amd/lib/var/*.so; do
  n=$(basename $lib .so)
  NORI_GPU_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/var_$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  grep '^{' gpurun_out/var_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(' ', round(d['value'],1), d['wavefront_iterations'], {k: round(v,2) for k,v in d['kernel_ms'].items()})"
done
# the default library with the film splat serialised after the finisher
NORI_SPLAT_OVERLAP=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/var_nooverlap.log 2>&1
rc=$?; echo "no-overlap rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
grep '^{' gpurun_out/var_nooverlap.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(' ', round(d['value'],1), d['wavefront_iterations'], {k: round(v,2) for k,v in d['kernel_ms'].items()})"
