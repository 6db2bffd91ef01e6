#!/bin/bash
# rocprofv3 on the bench command: one kernel-trace/stats run, then one PMC pass per
# TCC counter (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  No --pmc run
# is combined with a trace domain.  Outputs under gpurun_out/prof_<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
ARGS=${PROF_BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline --check 0"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE ${EXTRA_PMC:-}; do
  timeout -k 10 300 rocprofv3 --pmc ${C//,/ } --output-format csv -d $OUT/pmc_$C -o run -- python3 bench.py $ARGS > $OUT/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_$C.log; exit $rc; }
done
python3 tools/prof_summary.py $OUT $TAG "$ARGS"
