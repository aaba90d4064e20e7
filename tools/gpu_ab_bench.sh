#!/bin/bash
# Interleaved A/B of the headline bench over library builds (NORI_GPU_LIB):
# each argument is a library path under nori-ray-tracer_amd/lib ("-" = default).
# usage: REPS=2 tools/gpu_ab_bench.sh lib/libnori_gpu_base.so -
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
reps=${REPS:-2}
for r in $(seq 1 $reps); do
  for l in "$@"; do
    if [ "$l" = "-" ]; then unset NORI_GPU_LIB; else export NORI_GPU_LIB=$PWD/nori-ray-tracer_amd/$l; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity > gpurun_out/ab_bench.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$l rc=$rc"; tail -3 gpurun_out/ab_bench.log; exit $rc; fi
    python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.log')); print('$l', round(d['value'],1), {k: round(v,1) for k,v in d['kernel_ms'].items()})"
  done
done
