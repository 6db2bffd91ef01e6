#!/bin/bash
# concurrency test sensitivity (SLP build must fail, shipped build pass), window parity, window A/B
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06i}
mkdir -p "$out"
MV_LIB=build_variants/libmaveric_pose_slp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pose_concurrency.py -q --timeout 240 --timeout-method thread > "$out/concurrency_slp_build.log" 2>&1
echo "slp-build concurrency test rc=$? (expected non-zero)"
grep -E "assert|differ|passed|failed" "$out/concurrency_slp_build.log" | head -6
timeout -k 10 600 python -u -m pytest tests/test_gpu_pose_concurrency.py tests/test_gpu_frontend.py tests/test_gpu_tracking_main.py tests/test_gpu_track.py -x -q --timeout 240 --timeout-method thread > "$out/pytest_win.log" 2>&1 || { tail -30 "$out/pytest_win.log"; exit 1; }
tail -2 "$out/pytest_win.log"
TAG=${TAG:-r06i}/abw ROUNDS=2 LIBS="maveric-slam_amd/libmaveric_hip.so build_variants/libmaveric_feold.so" bash tools/ab_window.sh
