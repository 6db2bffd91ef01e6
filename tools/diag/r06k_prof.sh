#!/bin/bash
# Round 6's committed profiles: the headline (one context, so that rocprof's per-launch durations
# are not inflated by overlapping launches), the SURVEY C1 near-threshold data, the window front-end.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
(while sleep 50; do date >> gpurun_out/heartbeat_prof; done) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
A="--steps 10 --warmup 2 --extra-steps 0 --score-steps 0 --window-steps 0 --no-cpu-baseline --check 0 --pipeline 1"
PROF_BENCH_ARGS="$A" bash tools/profile.sh r06k || exit 1
PROF_BENCH_ARGS="$A --noise 0.05" bash tools/profile.sh r06k_nt || exit 1
TAG=r06k_window bash tools/gpu_window_prof.sh || exit 1
