#!/bin/bash
# SQ + HBM counters of the C3 run (tools/c3_bench.py), one rocprofv3 pass per group.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for g in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS" "FETCH_SIZE" "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"; do
  d=gpurun_out/pmcsq_c3_$i
  mkdir -p $d
  timeout -k 10 400 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $d -o run -- python3 tools/c3_bench.py 512 32 > $d/log 2>&1
  rc=$?; echo "group $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
