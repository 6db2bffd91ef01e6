#!/bin/bash
# round 4, call e: A/B of the pipelined A phase (D_APIPE) and the packed-FMA quantisation (D_PKQ)
# against the shipping build, with their phase traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TRACES="${TRACES:-trace:0.01875 apipe_trace:0.01875}" bash tools/gpu_trace_exp.sh || exit $?
for f in gpurun_out/tx_*.log; do echo "== $f"; grep -A1 "in flight per us" $f | cut -c1-200; done
TESTS_FOR="${TESTS_FOR:-apipe}" VARIANTS="${VARIANTS:-ship apipe pkq}" AB_STEPS=20 AB_SCORE=5 bash tools/gpu_ab.sh
