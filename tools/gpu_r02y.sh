#!/bin/bash
# The 64-spp share (8-GPU strong-scaling share of C2): finisher statistics,
# finisher phase clocks (NORI_PROF_FINISH build), a kernel trace for
# tools/timeline.py, then A/B of the termination lookahead and finisher width.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=nori-ray-tracer_amd/lib
B="python bench.py --no-cpu-baseline --no-parity --no-roofline"
NORI_DEBUG=1 timeout -k 10 200 $B --spp 64 --steps 3 > gpurun_out/s64_debug.log 2>&1 || { tail -5 gpurun_out/s64_debug.log; exit 1; }
grep "\[nori\]" gpurun_out/s64_debug.log | tail -4
NORI_DEBUG=1 NORI_GPU_LIB=$PWD/$L/var/pf.so timeout -k 10 200 $B --spp 64 --steps 3 > gpurun_out/s64_pf.log 2>&1 || { tail -5 gpurun_out/s64_pf.log; exit 1; }
grep "\[nori\]" gpurun_out/s64_pf.log | tail -4
mkdir -p gpurun_out/prof_s64
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s64 -o run -- \
    python3 bench.py --no-cpu-baseline --no-parity --no-roofline --spp 64 --steps 3 > gpurun_out/prof_s64/bench.log 2>&1 || exit 1
python3 tools/timeline.py gpurun_out/prof_s64
ab() { t=$1; v=$2; shift 2
  env $E NORI_GPU_LIB=$PWD/$L/$v.so timeout -k 10 300 $B "$@" > gpurun_out/ab.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "$t $v rc=$r"; tail -3 gpurun_out/ab.log; exit $r; }
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t $v [$E]', round(d['value'],1), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  for E in "NORI_X=0" "NORI_LOOKAHEAD=2" "NORI_LOOKAHEAD=3"; do ab s64 libnori_gpu --spp 64 --steps 10; done
  E="NORI_X=0"
  for v in var/fw16k var/fw4k; do ab s64 $v --spp 64 --steps 10; done
done
for E in "NORI_X=0" "NORI_LOOKAHEAD=3"; do ab c2 libnori_gpu; done
E="NORI_X=0"; ab c2 var/fw16k
