#!/bin/bash
# Round-4 measurements: the f16 subnormal probe, k_q8d_match phase traces on the headline's and on
# SURVEY C1's descriptor noise (indices only and with scores), and the near-threshold PMC profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 60 ./tools/probe_f16 > gpurun_out/probe_f16.log 2>&1 || { cat gpurun_out/probe_f16.log; exit 3; }
cat gpurun_out/probe_f16.log | tail -3
for cfg in "0.01875 0" "0.05 0" "0.05 1"; do
  set -- $cfg
  MV_LIB=build_variants/libmaveric_trace.so TN=$1 TS=$2 timeout -k 10 120 python tools/trace_direct.py \
      > gpurun_out/trace_n$1_s$2.log 2>&1 || { tail -20 gpurun_out/trace_n$1_s$2.log; exit 4; }
  echo "== noise $1 scores $2"; head -6 gpurun_out/trace_n$1_s$2.log
done
if [ "${PROF_NT:-1}" = 1 ]; then
  PROF_BENCH_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --check 1 --pipeline 1 --noise 0.05 --extra-steps 0 --score-steps 0 --window-steps 0" \
      bash tools/profile.sh r04a_nt || exit 5
fi
