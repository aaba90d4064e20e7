#!/bin/bash
# Glass-chain A/B (NORI_PROF_GLASS builds @name): lone-lane ns per chord bounce and the 64-spp share.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/glass
L=$GRAFT_REPO_ROOT/nori-ray-tracer_amd/lib
for r in 1 2; do for v in $1; do
  NORI_GPU_LIB=$L/libnori_gpu_$v.so NORI_DEBUG=1 timeout -k 10 120 python bench.py --spp 64 --steps 6 --warmup 2 --no-roofline --no-parity --no-cpu-baseline > gpurun_out/glass/$v.log 2>&1 || exit 1
  echo "$v: $(grep 'glass chains' gpurun_out/glass/$v.log | tail -1) | s64 $(grep '^{' gpurun_out/glass/$v.log | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['value'],1))")"
done; done
