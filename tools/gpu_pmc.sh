#!/bin/bash
# HBM traffic counters, one rocprofv3 pass per counter (FETCH_SIZE, WRITE_SIZE).
# usage: tools/gpu_pmc.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
for ctr in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_${tag}_$ctr
  mkdir -p $d
  timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $d -o run -- \
      python3 bench.py --no-cpu-baseline --no-parity "$@" > $d/bench.log 2>&1
  rc=$?; echo "$ctr rc=$rc"; ls $d; if [ $rc -ne 0 ]; then exit $rc; fi
done
