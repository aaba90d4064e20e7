#!/bin/bash
# Interleaved A/B over environment settings on the C3 height field and the
# reference's table scene.  Each argument is a space-separated VAR=value list
# ("-" = defaults).  usage: REPS=2 tools/gpu_ab_env.sh "NORI_PT=0" "NORI_PT=1"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
reps=${REPS:-2}
for r in $(seq 1 $reps); do
  for cfg in "$@"; do
    e=""; [ "$cfg" != "-" ] && e="$cfg"
    env $e timeout -k 10 300 python tools/c3_bench.py 512 ${C3_SPP:-64} > gpurun_out/ab_c3.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "[$cfg] c3 rc=$rc"; tail -3 gpurun_out/ab_c3.log; exit $rc; fi
    python3 -c "import json; d=json.load(open('gpurun_out/ab_c3.log')); print('C3    [$cfg]', round(d['Msamples_per_s'],1), {k: round(v,1) for k,v in d['kernel_ms'].items()})"
    env $e timeout -k 10 300 python tools/scene_bench.py scenes/pa4/table/table_path_mis.xml ${TABLE_SPP:-128} > gpurun_out/ab_table.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "[$cfg] table rc=$rc"; tail -3 gpurun_out/ab_table.log; exit $rc; fi
    python3 -c "import json; d=json.load(open('gpurun_out/ab_table.log')); print('table [$cfg]', round(d['Msamples_per_s'],1), d['kernel_ms'])"
  done
done
