#!/bin/bash
# XCD-aware order of the busy finisher blocks in BVH scenes (var/fx.so,
# -DNORI_FINISH_XCD=1): parity with the variant, then table scene / C3 A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$PWD/nori-ray-tracer_amd/lib
NORI_GPU_LIB=$L/var/fx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_png.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_fx.log 2>&1
r=$?; echo "pytest fx rc=$r"; tail -1 gpurun_out/pytest_fx.log; [ $r -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_fx.log | head -5; exit $r; }
for rep in 1 2; do
for v in libnori_gpu var/fx; do
  NORI_GPU_LIB=$L/$v.so timeout -k 10 300 python tools/scene_bench.py scenes/pa4/table/table_path_mis.xml 128 > gpurun_out/table.log 2>&1 || { echo "table $v failed"; tail -3 gpurun_out/table.log; exit 1; }
  echo "table $v: $(grep '^{' gpurun_out/table.log)"
done
done
for v in libnori_gpu var/fx libnori_gpu var/fx; do
  NORI_GPU_LIB=$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --no-roofline --config c3 --steps 3 --warmup 1 > gpurun_out/ab.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $v', round(d['value'],1))"
done
