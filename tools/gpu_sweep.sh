#!/bin/bash
# GPU tests, then bench for several path-pool sizes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for pool in "$@"; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --pool $pool > gpurun_out/bench_pool_$pool.log 2>&1
  rc=$?; echo "pool $pool rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
