#!/bin/bash
# XCD-aware order of k_direct's work-groups (var/dx.so, -DNORI_DIRECT_XCD=1):
# photon-map and one-bounce parity with the variant, then the photon-gather
# workload (cbox_pmap 800x600 32 spp 1M photons) A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=$PWD/nori-ray-tracer_amd/lib
NORI_GPU_LIB=$L/var/dx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_photon_map.py tests/test_gpu_one_bounce.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_dx.log 2>&1
r=$?; echo "pytest dx rc=$r"; tail -1 gpurun_out/pytest_dx.log; [ $r -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_dx.log | head -5; exit $r; }
for rep in 1 2; do
for v in libnori_gpu var/dx; do
  NORI_GPU_LIB=$L/$v.so timeout -k 10 300 python tools/extras_workload.py > gpurun_out/extras.log 2>&1 || { echo "extras $v failed"; tail -3 gpurun_out/extras.log; exit 1; }
  echo "$v: $(grep photonmapper gpurun_out/extras.log)"
done
done
