#!/bin/bash
# Is this box susceptible (the probe), does the diagnosis tool see the SLP build differ, does the test?
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06h}
mkdir -p "$out"
FORMS=8,10 PARTNERS=solo,network SAMPLES=0 timeout -k 10 300 python -u tools/diag/pk_probe.py > "$out/pk_probe.log" 2>&1 || exit 1
grep -E "^form" "$out/pk_probe.log"
MV_LIB=build_variants/libmaveric_pose_slp.so STAGES=none,net ROUNDS=4 timeout -k 10 300 python -u tools/dbg_pose_interference.py > "$out/dbg_slp.log" 2>&1 || exit 1
cat "$out/dbg_slp.log" | grep concurrent
MV_LIB=build_variants/libmaveric_pose_slp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pose_concurrency.py -x -q --timeout 240 --timeout-method thread > "$out/concurrency_slp_build.log" 2>&1
echo "slp-build concurrency test rc=$? (expected non-zero)"
grep -E "assert|differ|passed|failed" "$out/concurrency_slp_build.log" | head -5
exit 0
