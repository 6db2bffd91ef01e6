#!/bin/bash
# k_q8t_match vs k_q8d_match on SuperPoint descriptors (tools/ab_real.py) + the traced phases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05}
for thr in ${THRS:-0.8}; do
THR=$thr timeout -k 10 200 python tools/ab_real.py >> gpurun_out/${TAG}_abr.jsonl 2>gpurun_out/${TAG}_abr_t.err || exit $?
THR=$thr MV_Q8_KERNEL=d timeout -k 10 200 python tools/ab_real.py >> gpurun_out/${TAG}_abr.jsonl 2>gpurun_out/${TAG}_abr_d.err || exit $?
THR=$thr MV_LIB=build_variants/libmaveric_trace.so timeout -k 10 200 python tools/ab_real.py >> gpurun_out/${TAG}_abr.jsonl 2>gpurun_out/${TAG}_abr_tr.err || exit $?
done
cat gpurun_out/${TAG}_abr.jsonl
