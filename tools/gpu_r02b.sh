#!/bin/bash
# Kernel timelines of the strong-scaling share (C2 at 64 spp) and the full C2
# render (rocprofv3 kernel trace), plus the C4 bench after the env-map search fix.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for spp in 64 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$spp -o run -- \
    python3 bench.py --spp $spp --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/tl_$spp.log 2>&1
  r=$?; echo "trace $spp rc=$r"; if [ $r -ne 0 ]; then exit $r; fi
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k envmap -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_env.log 2>&1
r=$?; echo "envmap parity rc=$r"; tail -3 gpurun_out/pytest_env.log; if [ $r -gt 1 ]; then exit $r; fi
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1
r=$?; echo "c4 rc=$r"; tail -c 400 gpurun_out/bench_c4.log; exit $r
