#!/bin/bash
# Strong-scaling rehearsal on one GPU: the per-rank share of the C2 frame at
# N = 1, 2, 4, 8 ranks (passes split: 512/N spp of the full 512x512 frame),
# timed by bench.py; predicted N-GPU value = frame samples / share time
# (the film reduction, ~0.1-0.2 ms over xGMI, is not included).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for n in 1 2 4 8; do
  spp=$((512 / n))
  timeout -k 10 300 python bench.py --spp $spp --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/rehearsal_$n.log 2>&1
  r=$?; [ $r -ne 0 ] && { echo "N=$n rc=$r"; exit $r; }
  grep '^{' gpurun_out/rehearsal_$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); n=$n
t=d['ms_per_step']; print(f'N={n} share {d[\"config\"][\"workload\"]}: {t:.2f} ms/step, pool {d[\"config\"][\"path_pool\"]}, predicted {134217728/t/1e3:.0f} Msamples/s on {n} GPUs')"
done
