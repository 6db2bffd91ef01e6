#!/bin/bash
# round 4, call i: SuperPoint 64-channel layers' LDS staging without bank conflicts -- parity
# tests, the front-end bench against the previous build (spold), LDS / VALU / MFMA counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_superpoint.py tests/test_gpu_image_to_pose.py -m gpu -q -x \
    --timeout 200 --timeout-method thread > gpurun_out/sp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/sp_tests.log; [ $rc -eq 0 ] || exit $rc
lib() { [ "$1" = ship ] && echo maveric-slam_amd/libmaveric_hip.so || echo build_variants/libmaveric_$1.so; }
for rep in 1 2; do
  for v in spold ship; do
    MV_LIB=$(lib $v) timeout -k 10 200 python tools/bench_superpoint.py --batch 64 --steps 20 --check 1 > gpurun_out/sp_${v}_$rep.log 2>&1
    rc=$?; echo "sp $v rep $rep rc=$rc: $(tail -1 gpurun_out/sp_${v}_$rep.log | cut -c1-330)"
    [ $rc -eq 0 ] || exit $rc
  done
done
PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
    bash tools/prof_cmd.sh r04sp tools/bench_superpoint.py --batch 64 --steps 5 --check 0
