#!/bin/bash
# round 4, call f: the pair exchange with the deeper pipeline (import at the end of the tile, 4
# exchange / ring slots): tests on the exchange and forced-SOLO builds, A/B against the shipping
# build, phase traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TESTS_FOR="${TESTS_FOR:-xch xsolo}" VARIANTS="${VARIANTS:-ship xch}" AB_STEPS=20 AB_SCORE=5 \
    bash tools/gpu_ab.sh || exit $?
TRACES="${TRACES:-xch_trace:0.01875}" bash tools/gpu_trace_exp.sh || exit $?
