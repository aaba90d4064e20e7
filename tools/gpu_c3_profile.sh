#!/bin/bash
# Config C3 (tools/c3_bench.py): timing run, kernel trace + stats, and HBM /
# L2 / SQ counter passes (one rocprofv3 run per counter group), each under its
# own time limit.  NORI_POOL_PARTS=1 isolates the kernels (no stream overlap).
# usage: tools/gpu_c3_profile.sh <tag> [spp]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=${1:-c3}; spp=${2:-32}
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 300 python3 tools/c3_bench.py 512 128 > $o/bench.json 2> $o/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python3 tools/c3_bench.py 512 $spp > $o/trace.log 2>&1 || exit $?
i=0
for g in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"; do
  timeout -s KILL 300 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $o/pmc$i -o run -- python3 tools/c3_bench.py 512 $spp > $o/pmc$i.log 2>&1
  rc=$?; echo "pmc group $i ($g) rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
