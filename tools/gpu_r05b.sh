#!/bin/bash
# rocprofv3 kernel traces of the variants (which kernels ran, their durations).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
for v in "bin:-" "scan:NORI_EXTEND_BIN=0" "c3w8:NORI_BVH_WIDTH=8" "c3w4:-"; do
  tag=${v%%:*}; e=${v#*:}; [ "$e" = "-" ] && e=""
  args="--steps 2 --warmup 1 --no-cpu-baseline --no-parity"
  case $tag in c3*) args="$args --config c3";; esac
  env $e NORI_DEBUG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
      python3 bench.py $args > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  f=$(find $O/$tag -name "run_kernel_stats.csv" | head -1)
  echo "== $tag"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.2f} total_ms {float(r["TotalDurationNs"])/1e6:9.2f}')
PY
  grep -E "BVH|scan list|nodes" $O/$tag.log | head -3
done
