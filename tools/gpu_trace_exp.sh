#!/bin/bash
# k_q8d_match phase traces of several traced builds (build_variants/libmaveric_<name>.so, built
# on the CPU with -DMV_TRACE [+ timing-experiment switches]): per-wave A / sweep / epilogue cycles.
# TRACES: "name:noise[:scores] ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in ${TRACES:-trace:0.01875}; do
  IFS=: read name nz sc <<< "$spec"
  MV_LIB=build_variants/libmaveric_$name.so TN=$nz TS=${sc:-0} timeout -k 10 120 python tools/trace_direct.py \
      > gpurun_out/tx_${name}_n${nz}_s${sc:-0}.log 2>&1
  rc=$?
  echo "== $name noise $nz scores ${sc:-0} rc=$rc"; sed -n 2,6p gpurun_out/tx_${name}_n${nz}_s${sc:-0}.log
  [ $rc -eq 0 ] || exit $rc
done
