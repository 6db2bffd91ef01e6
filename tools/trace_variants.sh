#!/bin/bash
# k_i8_match loop anatomy: rebuild with the phase trace plus each ablation in VARIANTS
# (';'-separated compile flags) and print the per-tile loop cycles.  Timing only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS:-}"
i=0
for V in "${VS[@]}"; do
  touch maveric-slam_amd/csrc/hip/${VFILE:-k_allpairs_i8}.hip
  make -s -C maveric-slam_amd/csrc -j16 EXTRA="${TRACE_FLAG:--DI8_EXP_TRACE} $V" > gpurun_out/tv_$i.build 2>&1 || { echo "build failed: $V"; exit 2; }
  timeout -k 10 200 python ${TRACE:-tools/trace_i8.py} > gpurun_out/tv_$i.log 2>&1
  rc=$?
  echo "[$V] rc=$rc $(grep -E "per (64-col )?tile" gpurun_out/tv_$i.log) $(grep -E "^  (loop|sweep) " gpurun_out/tv_$i.log)"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
touch maveric-slam_amd/csrc/hip/${VFILE:-k_allpairs_i8}.hip
make -s -C maveric-slam_amd/csrc -j16 > /dev/null 2>&1
