#!/bin/bash
# Packed-FP32 two-ray scan: parity suite, then A/B on C2 (default = packed
# extension; nopack; packed shadow K=2) at 512 and 64 spp.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_png.py tests/test_table_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_par.log 2>&1
r=$?; echo "parity rc=$r"; tail -1 gpurun_out/pytest_par.log; [ $r -ne 0 ] && exit $r
NORI_GPU_LIB=$PWD/$L/var/sh2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_par_sh2.log 2>&1
r=$?; echo "parity sh2 rc=$r"; tail -1 gpurun_out/pytest_par_sh2.log; [ $r -ne 0 ] && exit $r
ab() { # tag lib args...
  t=$1; v=$2; shift 2
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v', round(d['value'],1), round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
}
for rep in 1 2; do for spp in 512 64; do
  ab s$spp libnori_gpu --spp $spp; ab s$spp var/nopack --spp $spp; ab s$spp var/sh2 --spp $spp
done; done
