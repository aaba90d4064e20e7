#!/bin/bash
# Full GPU suite (ABI 5: image textures / normal maps), then the C2 bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
r=$?; echo "pytest rc=$r"; grep -E "textured|passed|failed|Error" gpurun_out/pytest_gpu.log | tail -8; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/bench_c2.log 2>&1
r=$?; echo "bench rc=$r"; tail -c 300 gpurun_out/bench_c2.log; exit $r
