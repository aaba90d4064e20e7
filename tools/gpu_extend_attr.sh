#!/bin/bash
# Issue-slot attribution of the scan-mode extension kernel (k_extend_scan) on
# the roofline render of bench.py (one pool part, kernels serialised): the
# counters rocprofv3 can collect here and SQ counter passes of the default
# library (the round-5 NORI_PROF_EXTEND stamp build is gone; a
# lib/libnori_gpu_prof.so, if present, is run with NORI_DEBUG).  Every step
# has its own time limit; the script stops at the first failure.
# usage: tools/gpu_extend_attr.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/attr_$tag; mkdir -p $out
timeout -s KILL 60 rocprofv3 --list-avail > $out/avail.txt 2>&1
echo "list-avail rc=$?"
i=0
IFS=';' read -ra groups <<< "${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH}"
for g in "${groups[@]}"; do
  d=gpurun_out/pmcsq_attr_${tag}_$i; mkdir -p $d
  timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $d -o run -- \
      python3 bench.py --roofline-only "$@" > $d/bench.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
if [ -f nori-ray-tracer_amd/lib/libnori_gpu_prof.so ]; then
  NORI_DEBUG=1 NORI_GPU_LIB=$GRAFT_REPO_ROOT/nori-ray-tracer_amd/lib/libnori_gpu_prof.so \
    timeout -k 10 200 python3 bench.py --roofline-only "$@" > $out/prof.log 2>&1
  rc=$?; echo "stamp build rc=$rc"; grep "clocks per wave" $out/prof.log | tail -2
fi
python3 tools/pmc_summary.py attr_$tag > $out/summary.txt 2>&1; echo "summary rc=$?"; cat $out/summary.txt
exit 0
