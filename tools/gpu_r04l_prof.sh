#!/bin/bash
# round 4, the per-column-window build: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes
# over the headline command and over the SURVEY C1-noise command (bench.py --noise 0.05)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BASE="--steps 10 --warmup 2 --no-cpu-baseline --score-steps 0 --extra-steps 0 --window-steps 0 --pipeline 1"
T=${PTAG:-r04l}
PROF_BENCH_ARGS="$BASE --check 0" bash tools/profile.sh $T || exit $?
PROF_BENCH_ARGS="$BASE --check 1 --noise 0.05" bash tools/profile.sh ${T}_nt
