#!/bin/bash
# End-of-round check at HEAD: full GPU suite, smoke, the default bench line and
# the C3/C4/C5 lines, then the committed profiles of the C2 roofline render
# (kernel trace + stats, FETCH_SIZE / WRITE_SIZE and SQ counter passes).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
r=$?; echo "pytest rc=$r"; tail -1 gpurun_out/pytest_gpu.log; [ $r -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -5; exit $r; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench_c2.log; exit 1; }
grep '^{' gpurun_out/bench_c2.log
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 > gpurun_out/bench_$c.log 2>&1 || { echo bench $c failed; tail -5 gpurun_out/bench_$c.log; exit 1; }
  grep '^{' gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value'],1), d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --spp 64 --steps 10 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/bench_s64.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_s64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('s64', round(d['value'],1), d['ms_per_step'])"
tools/gpu_profile_all.sh r02 --roofline-only
