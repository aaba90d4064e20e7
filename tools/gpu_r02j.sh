#!/bin/bash
# Adaptive path pool (default) vs conditional shade loads, at 64/128/512 spp;
# kernel timeline of the 64-spp render.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
ab() { # tag lib args...
  t=$1; v=$2; shift 2
  NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v', round(d['value'],1), round(d['ms_per_step'],2), d['config']['path_pool'], d['wavefront_iterations'], {k:(round(v['avg_launch_ms'],4), round(v['frac'],3)) for k,v in d['roofline']['kernels'].items()})"
}
for rep in 1 2; do for spp in 64 128 512; do
  ab s$spp libnori_gpu --spp $spp; ab s$spp var/condload --spp $spp
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_64 -o run -- \
    python3 bench.py --spp 64 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/tl_64.log 2>&1
echo "trace rc=$?"
