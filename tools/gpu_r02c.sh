#!/bin/bash
# Parity of the traversal/shade path, the C2 bench, kernel timelines of the
# strong-scaling share (64 spp) and the full render, then the committed
# profile passes (kernel trace + stats, HBM counters, SQ counters) of
# `bench.py --roofline-only`.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${TAG:-r02}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_png.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_par.log 2>&1
r=$?; echo "parity rc=$r"; tail -2 gpurun_out/pytest_par.log; if [ $r -ne 0 ]; then exit $r; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1
r=$?; echo "bench rc=$r"; if [ $r -ne 0 ]; then exit $r; fi
for spp in 64 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_$spp -o run -- \
    python3 bench.py --spp $spp --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/tl_$spp.log 2>&1
  r=$?; echo "trace $spp rc=$r"; if [ $r -ne 0 ]; then exit $r; fi
done
[ -n "$NO_PROFILE" ] && exit 0
tools/gpu_profile_all.sh $tag --roofline-only
