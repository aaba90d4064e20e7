#!/bin/bash
# SQ instruction-mix counters for every kernel of one bench render: one
# rocprofv3 pass per counter group (groups separated by ';' in $PMC_GROUPS).
# usage: PMC_GROUPS="A B C;D E F" tools/gpu_pmc_sq.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
IFS=';' read -ra groups <<< "${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE}"
i=0
for g in "${groups[@]}"; do
  d=gpurun_out/pmcsq_${tag}_$i
  mkdir -p $d
  timeout -k 10 400 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $d -o run -- \
      python3 bench.py --no-cpu-baseline --no-parity "$@" > $d/bench.log 2>&1
  rc=$?; echo "group $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
