#!/bin/bash
# Round-2 full GPU suite (incl. the compiled C++ adapter), smoke, bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
r=$?; echo "pytest rc=$r"; tail -1 gpurun_out/pytest_gpu.log; grep -E "adapter" gpurun_out/pytest_gpu.log | head -3; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
r=$?; echo "smoke rc=$r"; tail -2 gpurun_out/smoke.log; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1
r=$?; echo "bench rc=$r"; tail -c 400 gpurun_out/bench_c2.log; exit $r
