#!/bin/bash
# Interleaved A/B benchmark: each configuration (an env assignment, "-" = none)
# runs once per round for $REPS rounds; prints every value and the median.
# "@name" = NORI_GPU_LIB=<lib>/libnori_gpu_name.so (a variant build).
# usage: REPS=3 tools/gpu_ab.sh "- NORI_POOL_PARTS=1 NORI_POOL_PARTS=3,NORI_X=1 @variant" [bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/nori-ray-tracer_amd/lib
cfgs=""
for c in $1; do case $c in @*) c="NORI_GPU_LIB=$L/libnori_gpu_${c#@}.so";; esac; cfgs="$cfgs $c"; done
shift
reps=${REPS:-3}
for r in $(seq 1 $reps); do
  for c in $cfgs; do
    if [ "$c" = "-" ]; then envs=""; else envs="${c//,/ }"; fi  # a,b: two assignments
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/ab.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$c rc=$rc"; tail -3 gpurun_out/ab.log; exit $rc; fi
    v=$(grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['value'],1))")
    grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()).get('roofline') or {}; print('   roofline frac', round(r.get('frac', 0), 4), {k: round(v['avg_launch_ms'], 4) for k, v in (r.get('kernels') or {}).items()}, {k: round(v, 3) for k, v in (r.get('tail') or {}).items()})"
    echo "$c $v" | tee -a gpurun_out/ab_results.txt
    grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; k=json.loads(sys.stdin.read()).get('kernel_ms',{}); print('   kernel_ms', {a: round(b,2) for a,b in k.items()})"
  done
done
python3 - <<'PY'
import collections, statistics
d = collections.defaultdict(list)
for l in open("gpurun_out/ab_results.txt"):
    k, v = l.split()
    d[k].append(float(v))
for k, v in d.items():
    print(f"{k:28s} median {statistics.median(v):8.1f}  all {v}")
PY
