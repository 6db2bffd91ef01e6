#!/bin/bash
# the A phase with 3 register sets (2 batches of row quads in flight beside the one quantised) vs 2
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
MV_LIB=build_variants/libmaveric_aps3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_allpairs.py -x -q -k "f32 or allpairs" --timeout 240 --timeout-method thread > gpurun_out/r06gg_pytest.log 2>&1 || { tail -20 gpurun_out/r06gg_pytest.log; exit 1; }
tail -1 gpurun_out/r06gg_pytest.log
TAG=r06gg ROUNDS=3 LIBS="build_variants/libmaveric_aps3.so maveric-slam_amd/libmaveric_hip.so" bash tools/ab_libs.sh
