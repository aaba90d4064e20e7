# interleaved A/B of the C3 (BVH walk) path pool: 2M (default) against 4M / 6M / 8M
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
 for knob in NONE=1 NORI_PATH_POOL=4194304 NORI_PATH_POOL=6291456 NORI_PATH_POOL=8388608; do
  v=$(env $knob timeout -k 10 150 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-roofline 2>>gpurun_out/c3p.err | grep '^{' | python -c "import json,sys;print(round(json.loads(sys.stdin.read())['value'],1))")
  echo "rep=$r c3 $knob value=$v" | tee -a gpurun_out/c3p.log
 done
done
