#!/bin/bash
# rocprofv3 over an arbitrary python tool: one kernel-trace/stats run, then one PMC pass per
# counter group (groups ';'-separated in PMC, each within the gfx950 per-pass slot limits).
# No --pmc run is combined with a trace domain.  Usage: tools/prof_cmd.sh TAG script.py args...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 "$@" > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 $OUT/trace.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
IFS=';' read -ra GS <<< "${PMC:-FETCH_SIZE}"
i=0
for G in "${GS[@]}"; do
  timeout -k 10 120 rocprofv3 --pmc $G --output-format csv -d $OUT/pmc_$i -o run -- python3 "$@" > $OUT/pmc_$i.log 2>&1
  rc=$?; echo "pmc [$G] rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_$i.log; exit $rc; }
  i=$((i+1))
done
python3 tools/prof_summary.py $OUT $TAG "$*" > $OUT/summary.log; cat $OUT/summary.log | python3 -c "import json,sys; d=json.load(sys.stdin); [print(k, {a:round(b,3) for a,b in v.items()}) for k,v in d[\"kernels\"].items()]"
