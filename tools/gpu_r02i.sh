#!/bin/bash
# A/B: scan extension K=2 (default) vs K=4, shadow K=2 on C2; BVH trace kernels
# at 8 waves/SIMD on C3.  Each line: value, isolated per-launch ms and frac.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
ab() { # tag lib args...
  t=$1; v=$2; shift 2
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v', round(d['value'],1), round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
}
for rep in 1 2; do
  ab c2 libnori_gpu; ab c2 var/k4; ab c2 var/sh2
done
for rep in 1 2; do
  ab c3 libnori_gpu --config c3 --steps 3 --warmup 1; ab c3 var/tw8 --config c3 --steps 3 --warmup 1
done
