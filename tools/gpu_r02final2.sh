#!/bin/bash
# End-of-round check after the XCD-aware BVH walks: full GPU suite, smoke,
# bench lines (C2, C3, C4, C5, the 64-spp share), the C3 roofline-render
# profiles (trace + FETCH/WRITE + SQ passes) and one L2 hit/miss pass on C3.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
r=$?; echo "pytest rc=$r"; tail -1 gpurun_out/pytest_gpu.log; [ $r -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -5; exit $r; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench_c2.log; exit 1; }
grep '^{' gpurun_out/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', round(d['value'],1), d['roofline']['frac'], d['cpu_baseline']['value'])"
for c in c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 > gpurun_out/bench_$c.log 2>&1 || { echo bench $c failed; tail -5 gpurun_out/bench_$c.log; exit 1; }
  grep '^{' gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value'],1), d['roofline']['frac'], d['cpu_baseline']['value'])"
done
timeout -k 10 300 python bench.py --spp 64 --steps 10 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/bench_s64.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_s64.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('s64', round(d['value'],1), d['ms_per_step'])"
tools/gpu_profile_all.sh r02_c3 --config c3 --roofline-only || exit 1
d=gpurun_out/l2_c3; mkdir -p $d
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $d -o run -- \
    python3 bench.py --no-cpu-baseline --no-parity --config c3 --roofline-only > $d/bench.log 2>&1
echo "l2 pass rc=$?"
