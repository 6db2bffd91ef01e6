#!/bin/bash
# rocprofv3 of the secondary rows: kernel traces of the int8 all-pairs and windowed front-end
# benches, then ONE counter pass on the int8 bench (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE:
# the MFMA units' busy fraction).  No counter pass is combined with a trace domain.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02}
OUT=gpurun_out/prof_sec_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/i8 -o run -- python3 tools/bench_i8.py --cpu-seconds 0 --check 0 > $OUT/i8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/win -o run -- python3 tools/bench_window.py --cpu-seconds 0 --check 0 > $OUT/win.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/i8_pmc -o run -- python3 tools/bench_i8.py --cpu-seconds 0 --check 0 > $OUT/i8_pmc.log 2>&1 || exit $?
echo done
