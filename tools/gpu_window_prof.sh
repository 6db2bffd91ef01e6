#!/bin/bash
# rocprofv3 of the windowed int8 front-end (tools/bench_window.py, the bench's window_frontend line):
# kernel trace + FETCH/WRITE bytes + VALU/LDS/wave counters, each PMC group a pass of its own.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06ix_window}
PMC="FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  bash tools/prof_cmd.sh $TAG tools/bench_window.py --batch 8192 --steps 10 --warmup 2 --check 1 --cpu-seconds 0
