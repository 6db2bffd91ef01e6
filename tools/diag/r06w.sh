#!/bin/bash
# window parity + A/B (the branch-free fold in the round-5 loop vs the round-5 kernel)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06w}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_tracking_main.py tests/test_gpu_track.py -x -q --timeout 240 --timeout-method thread > "$out/pytest_win.log" 2>&1 || { tail -30 "$out/pytest_win.log"; exit 1; }
tail -2 "$out/pytest_win.log"
TAG=${TAG:-r06w}/abw ROUNDS=2 LIBS="maveric-slam_amd/libmaveric_hip.so build_variants/libmaveric_wincur.so" bash tools/ab_window.sh
