#!/bin/bash
# A/B bench runs: every library under nori-ray-tracer_amd/lib/var, then the
# default library under each environment setting given in $VARIANT_ENVS
# (space-separated, e.g. "NORI_FUSED_EXTEND=0 NORI_SPLAT_OVERLAP=0").
# usage: VARIANT_ENVS="..." tools/gpu_variants.sh [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
summ() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(' ', round(d['value'],1), d['wavefront_iterations'], {k: round(v,2) for k,v in (d.get('kernel_ms_isolated') or {}).items()})"; }
for lib in nori-ray-tracer_amd/lib/libnori_gpu.so nori-ray-tracer_amd/lib/var/*.so; do
  [ -f "$lib" ] || continue
  n=$(basename $lib .so)
  NORI_GPU_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/var_$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  summ gpurun_out/var_$n.log
done
for ev in $VARIANT_ENVS; do
  env "$ev" timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/var_$ev.log 2>&1
  rc=$?; echo "$ev rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  summ gpurun_out/var_$ev.log
done
