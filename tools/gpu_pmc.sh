#!/bin/bash
# Counter passes over one command (PMC_CMD, run after `--`), one rocprofv3 --pmc run per
# counter set (PMC_SETS: ';'-separated), no trace domain in any of them; prints the kernels
# matching PMC_KERNEL per set.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${PMC_SETS}"
i=0
for S in "${SETS[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $S -d gpurun_out/pmc_$i -o run -- $PMC_CMD > gpurun_out/pmc_$i.log 2>&1
  rc=$?; echo "set $i [$S] rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_$i.log; exit $rc; }
  python3 tools/prof_db.py gpurun_out/pmc_$i/run_results.db | grep "${PMC_KERNEL:-.}" || true
  i=$((i+1))
done
