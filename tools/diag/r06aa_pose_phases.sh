#!/bin/bash
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
MV_LIB=build_variants/libmaveric_pst.so timeout -k 10 120 python -u tools/diag/pose_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== noisy"
POSE_NOISE=1 MV_LIB=build_variants/libmaveric_pst.so timeout -k 10 120 python -u tools/diag/pose_phases.py 2>&1 | grep -v amdgpu.ids
