#!/bin/bash
# exact-fit pose starts at the scale floor: the pose tests, then an ABAB headline A/B against the
# previous build (pose ms per step, value)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06o}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest $(grep -ln "pose_from_matches\|pose_params" tests/test_gpu_*.py | tr "\n" " ") -x -q --timeout 240 --timeout-method thread > "$out/pytest_pose.log" 2>&1 || { tail -30 "$out/pytest_pose.log"; exit 1; }
tail -2 "$out/pytest_pose.log"
TAG=${TAG:-r06o}/ab ROUNDS=2 LIBS="maveric-slam_amd/libmaveric_hip.so build_variants/libmaveric_i8old.so" ARGS="--steps 20 --warmup 3 --no-cpu-baseline --check 1 --extra-steps 0 --window-steps 0 --score-steps 0" bash tools/ab_libs.sh
