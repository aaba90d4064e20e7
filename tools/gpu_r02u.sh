#!/bin/bash
# Kernel timeline of the 64-spp share (the 8-GPU strong-scaling rank) and of
# the 512-spp frame: where the fixed per-render time goes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for s in 64 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl_$s -- python3 bench.py --no-cpu-baseline --no-parity --spp $s --steps 3 --warmup 2 > gpurun_out/tl_$s.log 2>&1 || { echo "spp $s rc=$?"; tail -5 gpurun_out/tl_$s.log; exit 1; }
  grep '^{' gpurun_out/tl_$s.log | cut -c1-300
done
