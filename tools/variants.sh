#!/bin/bash
# Kernel-variant sweep on the GPU box: for each compile-flag set in VARIANTS (';'-separated,
# e.g. "-DAP_NBUF=4;-DAP_NBUF=8"), rebuild the library and run a short bench.  Each bench
# step has its own time limit; any failure ends the sweep.  Leaves the default build behind.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
BENCH=${BENCH:-bench.py}
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 3 --no-cpu-baseline --check 1"}
IFS=';' read -ra VS <<< "${VARIANTS:-}"
i=0
for V in "${VS[@]}"; do
  touch maveric-slam_amd/csrc/hip/${VFILE:-k_allpairs_f32}.hip
  make -s -C maveric-slam_amd/csrc -j16 EXTRA="$V" > gpurun_out/variant_$i.build 2>&1 || { echo "build failed: $V"; exit 2; }
  timeout -k 10 300 python $BENCH $ARGS > gpurun_out/variant_$i.log 2>&1
  rc=$?
  echo "variant $i [$V] rc=$rc: $(tail -1 gpurun_out/variant_$i.log | python3 -c 'import sys,json
try:
    d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("stages_ms_per_step", d.get("stages_ms")))
except Exception as e: print("no json", e)')"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
touch maveric-slam_amd/csrc/hip/${VFILE:-k_allpairs_f32}.hip
make -s -C maveric-slam_amd/csrc -j16 > /dev/null 2>&1
