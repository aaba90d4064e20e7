#!/bin/bash
# Scan-loop variants: branchless hit update (default), + software-pipelined
# scalar loads with groups of 2 / 1 triangles, against the previous build.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_par.log 2>&1
r=$?; echo "parity rc=$r"; tail -1 gpurun_out/pytest_par.log; [ $r -ne 0 ] && exit $r
for v in pipe2 pipe1; do
  NORI_GPU_LIB=$PWD/$L/var/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_par_$v.log 2>&1
  r=$?; echo "parity $v rc=$r"; tail -1 gpurun_out/pytest_par_$v.log; [ $r -ne 0 ] && exit $r
done
ab() { # tag lib args...
  t=$1; v=$2; shift 2
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v', round(d['value'],1), round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
}
for rep in 1 2; do
  for v in libnori_gpu var/old var/pipe2 var/pipe1; do ab s512 $v; done
done
for v in libnori_gpu var/old var/pipe2 var/pipe1; do ab s64 $v --spp 64; done
