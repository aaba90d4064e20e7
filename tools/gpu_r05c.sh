#!/bin/bash
# The persistent binned kernels: equivalence tests, counters against the per-lane scans, A/B, then the 8-wide BVH.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_extend_bin.py > gpurun_out/bin.log 2>&1; r=$?; echo "bin tests rc=$r: $(tail -1 gpurun_out/bin.log)"; [ $r -eq 0 ] || exit $r
rm -f gpurun_out/ab_results.txt
echo "== C2"; REPS=2 bash tools/gpu_ab.sh "NORI_EXTEND_BIN=0 - NORI_BIN_PERSIST=0" || exit 1
G="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY"
PMC_GROUPS="$G" timeout -k 10 600 bash tools/gpu_pmc_sq.sh r05bin --roofline-only || exit 1
NORI_EXTEND_BIN=0 PMC_GROUPS="$G" timeout -k 10 600 bash tools/gpu_pmc_sq.sh r05scan --roofline-only || exit 1
python3 tools/pmc_summary.py r05bin | grep -A20 -E "trace_bin|extend_scan|shadow_scan" | head -60
python3 tools/pmc_summary.py r05scan | grep -A20 -E "trace_bin|extend_scan|shadow_scan" | head -60
NORI_BVH_WIDTH=8 timeout -k 10 400 $PT tests/test_gpu_parity.py -k "bvh or large_mesh" > gpurun_out/w8.log 2>&1; r=$?; echo "8-wide parity rc=$r: $(tail -1 gpurun_out/w8.log)"; [ $r -eq 0 ] || exit $r
rm -f gpurun_out/ab_results.txt
echo "== C3"; REPS=2 bash tools/gpu_ab.sh "- NORI_BVH_WIDTH=8" --config c3 --steps 3 --warmup 1
