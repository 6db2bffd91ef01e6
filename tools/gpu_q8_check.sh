#!/bin/bash
# all-pairs parity tests (GPU), then a k_q8_match variant sweep on the bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_allpairs.py tests/test_two_way.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ap.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_ap.log; [ $rc -eq 0 ] || exit $rc
VFILE=k_allpairs_q8 VARIANTS="${VARIANTS:--DQ8_PF=0;-DQ8_PF=1;-DQ8_PF=2}" BENCH_ARGS="--steps 20 --warmup 3 --no-cpu-baseline --check 1 --score-steps 0 --extra-steps 0 --window-steps 0" bash tools/variants.sh
