#!/bin/bash
# Round 5, first measurement call: correctness of the new kernels, then A/B benches.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05a
O=gpurun_out/r05a
L=$GRAFT_REPO_ROOT/nori-ray-tracer_amd/lib
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_extend_bin.py > $O/bin.log 2>&1; r=$?; echo "bin tests rc=$r: $(tail -1 $O/bin.log)"; [ $r -eq 0 ] || exit $r
NORI_SPLAT2=1 timeout -k 10 400 $PT tests/test_gpu_parity.py -k "render_matches_oracle or headline" > $O/splat2.log 2>&1; r=$?; echo "splat2 parity rc=$r: $(tail -1 $O/splat2.log)"; [ $r -eq 0 ] || exit $r
NORI_BVH_WIDTH=8 timeout -k 10 400 $PT tests/test_gpu_parity.py -k "bvh or large_mesh" > $O/w8.log 2>&1; r=$?; echo "8-wide parity rc=$r: $(tail -1 $O/w8.log)"; [ $r -eq 0 ] || exit $r
rm -f gpurun_out/ab_results.txt
echo "== C2"; REPS=2 bash tools/gpu_ab.sh "NORI_EXTEND_BIN=0 - NORI_SHADOW_BIN=0 NORI_GPU_LIB=$L/libnori_gpu_nosph.so NORI_SPLAT2=1" || exit 1
rm -f gpurun_out/ab_results.txt
echo "== C3"; REPS=2 bash tools/gpu_ab.sh "- NORI_BVH_WIDTH=8" --config c3 --steps 3 --warmup 1 || exit 1
