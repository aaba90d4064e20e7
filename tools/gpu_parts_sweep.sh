#!/bin/bash
# Bench over pool parts (streams) x pool sizes: tools/gpu_parts_sweep.sh "1 2 3 4" "4194304 8388608"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
for parts in $1; do for pool in $2; do
  NORI_POOL_PARTS=$parts timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --pool $pool > gpurun_out/sw_${parts}_$pool.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "parts $parts pool $pool rc=$rc"; exit $rc; fi
  grep '^{' gpurun_out/sw_${parts}_$pool.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('parts $parts pool $pool', round(d['value'],1), d['wavefront_iterations'], round(d['kernel_ms']['wall'],2))"
done; done
