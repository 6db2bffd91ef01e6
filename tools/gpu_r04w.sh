#!/bin/bash
# round 4: MFMA-pipe busy cycles and the held clock of k_i8_match, shipping build and the
# fold-free timing build (I8_EXP_NOFOLD): one --pmc pass each (no trace domain)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ship i8nofold; do
  lib=maveric-slam_amd/libmaveric_hip.so; [ $v = ship ] || lib=build_variants/libmaveric_$v.so
  MV_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_i8_$v -o run \
      -- python3 tools/bench_i8.py --cpu-seconds 0 --check 0 --steps 20 > gpurun_out/pmc_i8_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_i8_$v.log; exit $rc; }
  python3 tools/prof_db.py gpurun_out/pmc_i8_$v/run_results.db | grep "k_i8_match" || true
done
