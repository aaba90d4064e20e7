#!/bin/bash
# Interleaved A/B of the C3 height-field config (tools/c3_bench.py) over
# library builds: each argument is a library path ("-" = the default build).
# usage: REPS=3 tools/gpu_ab_c3.sh lib/a.so - [N SPP via C3_ARGS]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
reps=${REPS:-3}
for r in $(seq 1 $reps); do
  for l in "$@"; do
    if [ "$l" = "-" ]; then unset NORI_GPU_LIB; else export NORI_GPU_LIB=$PWD/$l; fi
    timeout -k 10 300 python tools/c3_bench.py $C3_ARGS > gpurun_out/c3ab.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$l rc=$rc"; tail -3 gpurun_out/c3ab.log; exit $rc; fi
    python3 -c "import json,sys; d=json.load(open('gpurun_out/c3ab.log')); print('$l', round(d['Msamples_per_s'],1), {k: round(v,1) for k,v in d['kernel_ms'].items()})"
  done
done
