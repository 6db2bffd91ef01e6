#!/bin/bash
# round 4, call d: the pair exchange (k_q8d_match sweep_x, -DD_XCH=1) -- the all-pairs / pipeline
# tests on the exchange build and on the forced-SOLO build, A/B of the shipping build (no exchange)
# against the exchange (and the cooperative re-scores on top of it), phase traces with the chip-wide
# A-phase concurrency.  Every step under its own time limit; a failed step ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TESTS_FOR="${TESTS_FOR:-xch xsolo}" VARIANTS="${VARIANTS:-ship xch xcoop}" AB_STEPS=20 AB_SCORE=5 \
    bash tools/gpu_ab.sh || exit $?
TRACES="${TRACES:-trace:0.01875 xch_trace:0.01875 xskew_trace:0.01875}" bash tools/gpu_trace_exp.sh || exit $?
for f in gpurun_out/tx_*.log; do echo "== $f"; grep -A2 "in flight per us" $f | cut -c1-220; done
