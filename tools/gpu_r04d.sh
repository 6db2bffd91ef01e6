#!/bin/bash
# round 4, call d: the pair exchange (k_q8d_match sweep_x) -- the all-pairs / pipeline tests on
# the shipping build and on the forced-SOLO build, A/B against the build without the exchange
# (and the cooperative re-scores on top), then the int8 all-pairs bench with / without the
# packed dequantising FMAs.  Every step under its own time limit; a failed step ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TESTS_FOR="${TESTS_FOR:-ship xsolo}" VARIANTS="${VARIANTS:-noxch ship coop skew}" AB_STEPS=20 AB_SCORE=5 \
    bash tools/gpu_ab.sh || exit $?
TRACES="${TRACES:-trace:0.01875 noxch_trace:0.01875 skew_trace:0.01875 trace:0.05}" bash tools/gpu_trace_exp.sh || exit $?
for f in gpurun_out/tx_*.log; do echo "== $f"; grep -A2 "in flight per us" $f | cut -c1-200; done
lib() { [ "$1" = ship ] && echo maveric-slam_amd/libmaveric_hip.so || echo build_variants/libmaveric_$1.so; }
for rep in 1 2; do
  for v in ${I8_VARIANTS:-ship i8pk}; do
    MV_LIB=$(lib $v) timeout -k 10 200 python tools/bench_i8.py --cpu-seconds 0 --check 1 > gpurun_out/i8_${v}_$rep.log 2>&1
    rc=$?; echo "i8 $v rep $rep rc=$rc: $(tail -1 gpurun_out/i8_${v}_$rep.log | cut -c1-300)"
    [ $rc -eq 0 ] || exit $rc
  done
done
