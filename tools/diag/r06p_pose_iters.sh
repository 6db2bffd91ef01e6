#!/bin/bash
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for v in dg_head dg_floor dg_tight; do
  echo "== $v"
  MV_LIB=build_variants/libmaveric_$v.so timeout -k 10 120 python -u tools/diag/pose_iters.py 2>&1 | grep -v amdgpu.ids || exit 1
done
