#!/bin/bash
# k_i8_match variants (VARIANTS: ';'-separated compile-flag sets): per variant the int8 bench
# (pairs/s, stage times by HIP events); the default build restored at the end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
IFS=';' read -ra VS <<< "${VARIANTS:- }"
i=0
for V in "${VS[@]}"; do
  touch maveric-slam_amd/csrc/hip/k_allpairs_i8.hip
  make -s -C maveric-slam_amd/csrc -j16 EXTRA="$V" > gpurun_out/iv_$i.build 2>&1 || { echo "build failed: $V"; exit 2; }
  timeout -k 10 200 python tools/bench_i8.py --cpu-seconds 0 --check ${CHECK:-1} > gpurun_out/iv_$i.log 2>&1; rc=$?
  echo "variant $i [$V] rc=$rc: $(tail -1 gpurun_out/iv_$i.log | cut -c1-330)"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
touch maveric-slam_amd/csrc/hip/k_allpairs_i8.hip
make -s -C maveric-slam_amd/csrc -j16 > /dev/null 2>&1
