#!/bin/bash
# the one-pass int8 screen: all-pairs / two-way / pipeline / sequence parity (GPU), then a short
# headline bench.  Each GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest tests/test_gpu_allpairs.py tests/test_two_way.py tests/test_gpu_pipeline.py tests/test_gpu_sequence.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_direct.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_direct.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --check 2 --score-steps 5 --extra-steps 0 --window-steps 0"
IFS=';' read -ra VS <<< "${BENCH_VARIANTS:- ;--screen i8s}"
i=0
for V in "${VS[@]}"; do
  timeout -k 10 200 python bench.py $ARGS $V > gpurun_out/bench_d$i.log 2>&1; rc=$?
  echo "[$V] rc=$rc: $(tail -1 gpurun_out/bench_d$i.log | python3 -c 'import sys,json
try:
    d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stages_ms_per_step"], d["with_scores"])
except Exception as e: print("no json", e)')"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
