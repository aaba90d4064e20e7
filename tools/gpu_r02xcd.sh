#!/bin/bash
# XCD-aware block order for the BVH walks (var/xcd.so, -DNORI_XCD_REMAP=1):
# parity with the variant, then C3 and the table scene A/B against the default.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$PWD/nori-ray-tracer_amd/lib
NORI_GPU_LIB=$L/var/xcd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_png.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_xcd.log 2>&1
r=$?; echo "pytest xcd rc=$r"; tail -1 gpurun_out/pytest_xcd.log; [ $r -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_xcd.log | head -5; exit $r; }
B="python bench.py --no-cpu-baseline --no-parity --no-roofline"
ab() { t=$1; v=$2; shift 2
  NORI_GPU_LIB=$L/$v.so timeout -k 10 300 $B "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v', round(d['value'],1), round(d['ms_per_step'],3))"
}
for rep in 1 2 3; do
  for v in libnori_gpu var/xcd; do ab c3 $v --config c3 --steps 3 --warmup 1; done
done
for v in libnori_gpu var/xcd; do
  NORI_GPU_LIB=$L/$v.so timeout -k 10 300 python tools/scene_bench.py scenes/pa4/table/table_path_mis.xml 128 > gpurun_out/table_$(basename $v).log 2>&1 || { echo "table $v failed"; tail -3 gpurun_out/table_$(basename $v).log; exit 1; }
  echo "table $v: $(tail -n 2 gpurun_out/table_$(basename $v).log | tr '\n' ' ')"
done
for v in libnori_gpu var/xcd; do ab c2 $v; done
