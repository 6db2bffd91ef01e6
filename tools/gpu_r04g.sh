#!/bin/bash
# round 4, call g: where the exchange build's time goes -- phase traces of the exchange build,
# the same without its exchange-slot stores, and without its imports (timing experiments)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TRACES="${TRACES:-trace:0.01875 xch_trace:0.01875 xnost_trace:0.01875 xnoimp_trace:0.01875}" bash tools/gpu_trace_exp.sh || exit $?
for f in gpurun_out/tx_*trace_n0.01875_s0.log; do echo "== $f"; grep -h "real time" $f; done
