#!/bin/bash
# which change makes the round-5 window kernel agree with the oracle on the exact-tie case
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for lib in maveric-slam_amd/libmaveric_hip.so build_variants/libmaveric_v1.so build_variants/libmaveric_v3.so build_variants/libmaveric_v4.so; do
  echo "== $lib"
  MV_LIB=$lib timeout -k 10 120 python -u tools/diag/dbg_window_tie.py 2>&1 | grep -E "differing|matches" || exit 1
done
