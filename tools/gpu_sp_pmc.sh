#!/bin/bash
# SuperPoint per-layer counters: the kernel trace (per-dispatch durations) and two PMC passes
# over tools/bench_superpoint.py (batch 64), each pass its own rocprofv3 run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
CMD="python3 tools/bench_superpoint.py --batch 64 --steps 3 --warmup 1 --check 0"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/spk -o run -- $CMD > gpurun_out/spk.log 2>&1 || { echo trace failed; tail -5 gpurun_out/spk.log; exit 1; }
PMC_CMD="$CMD" PMC_KERNEL="k_sp" PMC_SETS="${PMC_SETS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES;SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS}" bash tools/gpu_pmc.sh
