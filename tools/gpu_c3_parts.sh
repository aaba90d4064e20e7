# interleaved A/B of C3's pool parts at the 4M path pool: 3 (default) against 2 / 4
set -e
mkdir -p gpurun_out
for r in 1 2; do
 for knob in NONE=1 NORI_POOL_PARTS=2 NORI_POOL_PARTS=4; do
  v=$(env $knob timeout -k 10 150 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-roofline 2>>gpurun_out/c3pp.err | grep '^{' | python -c "import json,sys;print(round(json.loads(sys.stdin.read())['value'],1))")
  echo "rep=$r c3 $knob value=$v" | tee -a gpurun_out/c3pp.log
 done
done
