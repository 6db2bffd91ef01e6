set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06it
for v in ${VARIANTS:-peel fold2}; do
  MV_LIB=build_variants/win/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d gpurun_out/r06it/$v -o run -- python3 tools/bench_window.py --batch 8192 --steps 3 --warmup 1 --check 0 --cpu-seconds 0 > gpurun_out/r06it/$v.log 2>&1 || exit $?
  python3 tools/prof_db.py gpurun_out/r06it/$v/run_results.db > gpurun_out/r06it/$v.txt 2>&1 || exit $?
done
