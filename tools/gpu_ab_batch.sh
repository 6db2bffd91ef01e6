#!/bin/bash
# k_q8t_match vs k_q8d_match over batch sizes (tools/ab_batch.py), each kernel in its own process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05}
timeout -k 10 200 python tools/ab_batch.py > gpurun_out/${TAG}_abb_t.jsonl 2>gpurun_out/${TAG}_abb_t.err || exit $?
MV_Q8_KERNEL=d timeout -k 10 200 python tools/ab_batch.py > gpurun_out/${TAG}_abb_d.jsonl 2>gpurun_out/${TAG}_abb_d.err || exit $?
cat gpurun_out/${TAG}_abb_t.jsonl gpurun_out/${TAG}_abb_d.jsonl
