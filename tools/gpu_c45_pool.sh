# interleaved A/B of the C4 / C5 path pool: 4M (default) against 2M / 8M
set -e
mkdir -p gpurun_out
for r in 1 2; do
 for cfg in c5 c4; do
  for knob in NONE=1 NORI_PATH_POOL=2097152 NORI_PATH_POOL=8388608; do
   v=$(env $knob timeout -k 10 150 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-roofline 2>>gpurun_out/c45p.err | grep '^{' | python -c "import json,sys;print(round(json.loads(sys.stdin.read())['value'],1))")
   echo "rep=$r $cfg $knob value=$v" | tee -a gpurun_out/c45p.log
  done
 done
done
