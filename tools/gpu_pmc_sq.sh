#!/bin/bash
# SQ instruction-mix counters for every kernel of one bench render (one rocprofv3 pass).
# usage: tools/gpu_pmc_sq.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
d=gpurun_out/pmcsq_${tag}
mkdir -p $d
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $d -o run -- \
    python3 bench.py --no-cpu-baseline --no-parity "$@" > $d/bench.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
