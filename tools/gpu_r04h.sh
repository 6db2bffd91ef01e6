#!/bin/bash
# round 4, call h: the exchange's imports -- from the partner's slot (xch), from the block's own
# slot (xown, same data volume, no cross-CU hand-off), one 16-B chunk (xnoimp); timing only
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TRACES="${TRACES:-xch_trace:0.01875 xown_trace:0.01875 xnoimp_trace:0.01875}" bash tools/gpu_trace_exp.sh
for f in gpurun_out/tx_x*_trace_n0.01875_s0.log; do echo "== $f"; grep -h "real time" $f; done
