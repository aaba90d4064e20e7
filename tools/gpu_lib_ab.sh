# interleaved A/B of the default library against a variant build (lib/libnori_gpu_$1.so) on C4, C5, C2
set -e
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/nori-ray-tracer_amd/lib
for r in 1 2 3; do
 for cfg in c5 c4 c2; do
  for lib in libnori_gpu.so libnori_gpu_$1.so; do
   v=$(NORI_GPU_LIB=$L/$lib timeout -k 10 150 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-roofline 2>>gpurun_out/lab.err | grep '^{' | python -c "import json,sys;print(round(json.loads(sys.stdin.read())['value'],1))")
   echo "rep=$r cfg=$cfg $lib value=$v" | tee -a gpurun_out/lab.log
  done
 done
done
