#!/bin/bash
# BVH traversal: stack top cached in registers (variant) vs default, C3 + table.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
NORI_GPU_LIB=$PWD/$L/var/topreg.so timeout -k 10 400 python -u -m pytest tests/test_table_golden.py tests/test_gpu_reference_png.py -k "table or large or c3 or height" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tr.log 2>&1
r=$?; echo "parity rc=$r"; tail -1 gpurun_out/pytest_tr.log; [ $r -ne 0 ] && exit $r
ab() { t=$1; v=$2; shift 2
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v', round(d['value'],1), round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
}
for rep in 1 2; do for v in libnori_gpu var/topreg; do ab c3 $v --config c3 --steps 3 --warmup 1; done; done
for v in libnori_gpu var/topreg; do
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python tools/scene_bench.py scenes/pa4/table/table_path_mis.xml 128 > gpurun_out/sb.log 2>&1; echo "table $v rc=$?"; tail -1 gpurun_out/sb.log
done
