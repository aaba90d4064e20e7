# interleaved A/B of the C3 (BVH walk) run-time knobs: path pool and LDS stack depth
set -e
mkdir -p gpurun_out
for r in 1 2; do
 for knob in NONE=1 NORI_PATH_POOL=1048576 NORI_PATH_POOL=3145728 NORI_PATH_POOL=4194304 NORI_BVH_STACK=32 NORI_POOL_PARTS=4; do
  v=$(env $knob timeout -k 10 150 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-roofline 2>>gpurun_out/c3k.err | grep '^{' | python -c "import json,sys;print(round(json.loads(sys.stdin.read())['value'],1))")
  echo "rep=$r c3 $knob value=$v" | tee -a gpurun_out/c3k.log
 done
done
