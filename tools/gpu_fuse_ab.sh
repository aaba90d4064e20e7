set -e
mkdir -p gpurun_out
for r in 1 2 3; do
 for cfg in c5 c4; do
  for f in 1 0; do
   v=$(NORI_TRACE_FUSE=$f timeout -k 10 120 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-roofline 2>>gpurun_out/ab.err | grep '^{' | python -c "import json,sys;print(round(json.loads(sys.stdin.read())['value'],1))")
   echo "rep=$r cfg=$cfg fuse=$f value=$v" | tee -a gpurun_out/ab.log
  done
 done
done
