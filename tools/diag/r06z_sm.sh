#!/bin/bash
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06z}
mkdir -p "$out"
for lib in build_variants/libmaveric_sm512.so build_variants/libmaveric_sm128.so; do
  MV_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -x -q --timeout 240 --timeout-method thread > "$out/pytest_$(basename $lib .so).log" 2>&1 || { tail -30 "$out/pytest_$(basename $lib .so).log"; exit 1; }
  tail -1 "$out/pytest_$(basename $lib .so).log"
done
TAG=${TAG:-r06z}/abw ROUNDS=2 LIBS="maveric-slam_amd/libmaveric_hip.so build_variants/libmaveric_sm512.so build_variants/libmaveric_sm128.so" bash tools/ab_window.sh
