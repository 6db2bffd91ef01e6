#!/bin/bash
# rocprofv3 of the headline command (one context, --pipeline 1: launch durations not inflated by
# overlap), headline descriptors and SURVEY C1's sigma 0.05: kernel trace, FETCH_SIZE, WRITE_SIZE,
# and the issue counters; then the same counters on k_q8d_match (MV_Q8_KERNEL=d) for the A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05d}
BASE="--steps 10 --warmup 2 --extra-steps 0 --score-steps 0 --window-steps 0 --no-cpu-baseline --check 0 --pipeline 1"
export EXTRA_PMC="SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_ANY GRBM_GUI_ACTIVE,SQ_VALU_MFMA_BUSY_CYCLES"
PROF_BENCH_ARGS="$BASE" bash tools/profile.sh ${TAG} > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
grep -A3 '"k_q8t_match"' gpurun_out/prof_${TAG}/summary_${TAG}.json | head -5
PROF_BENCH_ARGS="$BASE --noise 0.05" bash tools/profile.sh ${TAG}_nt > gpurun_out/${TAG}_nt_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_nt_prof.log; exit 1; }
if [ "${WITH_D:-1}" = 1 ]; then
  MV_Q8_KERNEL=d PROF_BENCH_ARGS="$BASE" bash tools/profile.sh ${TAG}_q8d > gpurun_out/${TAG}_q8d_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_q8d_prof.log; exit 1; }
fi
echo done
