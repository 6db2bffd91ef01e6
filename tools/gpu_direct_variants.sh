#!/bin/bash
# k_q8d_match variants (VARIANTS: ';'-separated compile-flag sets): per variant a short headline
# bench (kernel time by HIP events) and the phase trace; the default build restored at the end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --check ${CHECK:-1} --score-steps 0 --extra-steps 0 --window-steps 0"
IFS=';' read -ra VS <<< "${VARIANTS:- }"
i=0
for V in "${VS[@]}"; do
  touch maveric-slam_amd/csrc/hip/k_allpairs_direct.hip
  make -s -C maveric-slam_amd/csrc -j16 EXTRA="$V" > gpurun_out/dv_$i.build 2>&1 || { echo "build failed: $V"; exit 2; }
  timeout -k 10 200 python bench.py $ARGS > gpurun_out/dv_$i.log 2>&1; rc=$?
  echo "variant $i [$V] rc=$rc: $(tail -1 gpurun_out/dv_$i.log | python3 -c 'import sys,json
try:
    d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stages_ms_per_step"], d["roofline"]["frac"])
except Exception as e: print("no json", e)')"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/dv_$i.log; exit $rc; }
  if [ -n "${TRACE:-}" ]; then
    touch maveric-slam_amd/csrc/hip/k_allpairs_direct.hip
    make -s -C maveric-slam_amd/csrc -j16 EXTRA="-DMV_TRACE $V" > gpurun_out/dv_$i.tbuild 2>&1 || exit 2
    timeout -k 10 120 python tools/trace_direct.py > gpurun_out/dv_$i.trace 2>&1 || { tail -5 gpurun_out/dv_$i.trace; exit 3; }
    sed -n 2,9p gpurun_out/dv_$i.trace
  fi
  i=$((i+1))
done
touch maveric-slam_amd/csrc/hip/k_allpairs_direct.hip
make -s -C maveric-slam_amd/csrc -j16 > /dev/null 2>&1
