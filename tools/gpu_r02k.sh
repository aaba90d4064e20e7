#!/bin/bash
# Round-2 evidence in one call: GPU test suite, bench lines (C2 with CPU
# baseline + parity; the 64-spp strong-scaling share; C3, C4, C5), then the
# committed profile passes of `bench.py --roofline-only` (kernel trace +
# stats, FETCH_SIZE / WRITE_SIZE, SQ counters).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
r=$?; echo "pytest rc=$r"; tail -1 gpurun_out/pytest_gpu.log; [ $r -ne 0 ] && exit $r
b() { # name, args...
  n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/bench_$n.log 2>&1
  r=$?; echo "bench $n rc=$r"; return $r
}
b c2 && b c2spp64 --spp 64 --no-cpu-baseline --no-parity && \
b c3 --config c3 --steps 3 --warmup 1 --cpu-seconds 10 && \
b c4 --config c4 --steps 3 --warmup 1 --cpu-seconds 10 && \
b c5 --config c5 --steps 3 --warmup 1 --cpu-seconds 10 || exit 1
[ -n "$NO_PROFILE" ] && exit 0
tools/gpu_profile_all.sh ${TAG:-r02} --roofline-only
