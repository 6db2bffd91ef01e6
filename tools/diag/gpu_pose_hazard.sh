#!/bin/bash
# Round-6 diagnosis of k_pose_ransac's concurrency-dependent results, one GPU call:
#  (1) the pose beside the SuperPoint forward on another stream, for four builds of the pose object
#      only: shipped (-fno-slp-vectorize), SLP-packed (the round-5 -O3 build that misbehaved), SLP +
#      an s_nop before every instruction, SLP + every s_waitcnt forced to zero;
#  (2) the SLP build run SOLO after every CU's registers and LDS were filled with 4 patterns.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06a}
mkdir -p "$out"
for v in default slp pad wz; do
  lib=maveric-slam_amd/libmaveric_hip.so
  [ "$v" != default ] && lib=build_variants/libmaveric_pose_$v.so
  echo "== $v ($lib)" | tee -a "$out/summary.log"
  MV_LIB=$lib STAGES=none,net ROUNDS=${ROUNDS:-4} timeout -k 10 240 python -u tools/dbg_pose_interference.py \
      > "$out/conc_$v.log" 2>&1
  grep concurrent "$out/conc_$v.log" | tee -a "$out/summary.log"
done
for v in slp default; do
  lib=maveric-slam_amd/libmaveric_hip.so
  [ "$v" != default ] && lib=build_variants/libmaveric_pose_$v.so
  echo "== fill test $v" | tee -a "$out/summary.log"
  MV_LIB=$lib FILLTEST=1 ROUNDS=8 timeout -k 10 240 python -u tools/dbg_pose_interference.py > "$out/fill_$v.log" 2>&1
  grep fill "$out/fill_$v.log" | tee -a "$out/summary.log"
done
