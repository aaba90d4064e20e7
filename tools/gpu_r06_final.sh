#!/bin/bash
# Round-6 evidence: the GPU suite + smoke, bench lines of C2-C5 and the
# per-rank shares of the strong-scaling model (512/256/128/64 spp).
# Every step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-final6}
bash tools/gpu_suite.sh --configs "c2 c3 c4 c5" --tag $TAG || exit $?
for s in 256 128 64; do
  timeout -k 10 300 python bench.py --spp $s --steps 10 --no-cpu-baseline --no-parity --no-roofline > gpurun_out/$TAG/share_$s.log 2>&1 || exit 1
  grep '^{' gpurun_out/$TAG/share_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('spp $s', round(d['value'],1), round(d['ms_per_step'],3), 'ms')"
done
exit 0
