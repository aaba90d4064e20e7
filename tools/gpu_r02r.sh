#!/bin/bash
# Branch-free cooperative scan with the exact fast reciprocal: parity, then
# finisher profile (new vs old) and 64/512-spp benches.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_png.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_par.log 2>&1
r=$?; echo "parity rc=$r"; tail -1 gpurun_out/pytest_par.log; [ $r -ne 0 ] && exit $r
for v in proffin oldpf; do
  NORI_DEBUG=1 NORI_GPU_LIB=$PWD/$L/var/$v.so timeout -k 10 300 python bench.py --spp 64 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/pf_$v.log 2>&1
  r=$?; echo "$v rc=$r"; grep "finisher" gpurun_out/pf_$v.log | tail -2
done
ab() { t=$1; v=$2; shift 2
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v', round(d['value'],1), round(d['ms_per_step'],2))"
}
for rep in 1 2 3; do for v in libnori_gpu var/old; do ab s64 $v --spp 64 --steps 10 --warmup 3; done; done
for v in libnori_gpu var/old; do ab s512 $v; done
