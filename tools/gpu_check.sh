#!/bin/bash
# One gpurun call: GPU parity tests, then the bench (stops at the first crash/timeout).
# usage: tools/gpu_check.sh [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
