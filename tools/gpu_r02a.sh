#!/bin/bash
# Round 2, first GPU call: the GPU test suite, then the bench lines (C2 with
# CPU baseline and parity, the HIP-runtime A/B, the per-rank shares of a
# strong-scaled C2, C3/C4/C5).  Stops at the first crash/timeout.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "affinity $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null) nproc $(nproc)"
timeout -k 10 600 python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
b() { # name, args...
  n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/bench_$n.log 2>&1
  r=$?; echo "bench $n rc=$r"; tail -c 600 gpurun_out/bench_$n.log | tail -2; return $r
}
b c2 --steps 10 --warmup 3 && \
b c2spp64 --spp 64 --steps 10 --warmup 3 --no-cpu-baseline --no-parity && \
b c2spp128 --spp 128 --steps 10 --warmup 3 --no-cpu-baseline --no-parity && \
b c5 --config c5 --steps 3 --warmup 1 --cpu-seconds 8 && \
b c4 --config c4 --steps 3 --warmup 1 --cpu-seconds 8 && \
b c3 --config c3 --steps 3 --warmup 1 --cpu-seconds 8
