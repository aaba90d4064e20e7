# the GPU suite, then every config's bench line at the default trace-launch setting
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt2.log 2>&1
tail -2 gpurun_out/gt2.log
for r in 1 2; do
 for cfg in c5 c4 c3 c2; do
  v=$(timeout -k 10 150 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-roofline 2>>gpurun_out/fd.err | grep '^{' | python -c "import json,sys;print(round(json.loads(sys.stdin.read())['value'],1))")
  echo "rep=$r cfg=$cfg default value=$v" | tee -a gpurun_out/fd.log
 done
done
