# interleaved A/B of run-time knobs on the full-plugin configs (C4, C5)
set -e
mkdir -p gpurun_out
for r in 1 2; do
 for cfg in c5 c4; do
  for knob in NONE=1 NORI_POOL_PARTS=2 NORI_POOL_PARTS=4 NORI_RTC_K=2 NORI_FINISH_FIRST=0; do
   v=$(env $knob timeout -k 10 150 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-roofline 2>>gpurun_out/kn.err | grep '^{' | python -c "import json,sys;print(round(json.loads(sys.stdin.read())['value'],1))")
   echo "rep=$r cfg=$cfg $knob value=$v" | tee -a gpurun_out/kn.log
  done
 done
done
