#!/bin/bash
# round 4, call e: A/B of the exchange build against the exchange + first-wave skew (D_SKEW) and
# + pipelined A phase (D_APIPE) builds, the pipelined A phase's trace, and the int8 all-pairs bench
# with / without the packed dequantising FMAs (I8_PK).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TESTS_FOR="${TESTS_FOR:-apipe}" VARIANTS="${VARIANTS:-ship apipe}" AB_STEPS=20 AB_SCORE=0 \
    AB_NOISE=0.01875 bash tools/gpu_ab.sh || exit $?
TRACES="${TRACES:-apipe_trace:0.01875}" bash tools/gpu_trace_exp.sh || exit $?
lib() { [ "$1" = ship ] && echo maveric-slam_amd/libmaveric_hip.so || echo build_variants/libmaveric_$1.so; }
for rep in 1 2; do
  for v in ${I8_VARIANTS:-ship i8pk}; do
    MV_LIB=$(lib $v) timeout -k 10 200 python tools/bench_i8.py --cpu-seconds 0 --check 1 > gpurun_out/i8_${v}_$rep.log 2>&1
    rc=$?; echo "i8 $v rep $rep rc=$rc: $(tail -1 gpurun_out/i8_${v}_$rep.log | cut -c1-300)"
    [ $rc -eq 0 ] || exit $rc
  done
done
