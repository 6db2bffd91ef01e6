#!/bin/bash
# SuperPoint kernel variants (VARIANTS: ';'-separated compile-flag sets): per variant the
# front-end bench (frames/s, stage times by HIP events); the default build restored at the end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
IFS=';' read -ra VS <<< "${VARIANTS:- }"
i=0
for V in "${VS[@]}"; do
  touch maveric-slam_amd/csrc/hip/k_superpoint.hip
  make -s -C maveric-slam_amd/csrc -j16 EXTRA="$V" > gpurun_out/sv_$i.build 2>&1 || { echo "build failed: $V"; exit 2; }
  timeout -k 10 200 python tools/bench_superpoint.py --batch 64 --steps 10 --check ${CHECK:-1} > gpurun_out/sv_$i.log 2>&1; rc=$?
  echo "variant $i [$V] rc=$rc: $(tail -1 gpurun_out/sv_$i.log | cut -c1-260)"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
touch maveric-slam_amd/csrc/hip/k_superpoint.hip
make -s -C maveric-slam_amd/csrc -j16 > /dev/null 2>&1
