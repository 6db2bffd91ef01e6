#!/bin/bash
# Round-6 diagnosis, second call: (1) the packed-FP32 instruction probe alone and beside the network;
# (2) the pose beside the network for the SLP build with the 8-point QR kept scalar (and the shipped /
# SLP builds again on the same box as controls).
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06b}
mkdir -p "$out"
timeout -k 10 300 python -u tools/diag/pk_probe.py > "$out/pk_probe.log" 2>&1
cat "$out/pk_probe.log" | grep form | tee -a "$out/summary.log"
for v in qr slp default; do
  lib=maveric-slam_amd/libmaveric_hip.so
  [ "$v" != default ] && lib=build_variants/libmaveric_pose_$v.so
  echo "== $v ($lib)" | tee -a "$out/summary.log"
  MV_LIB=$lib STAGES=none,net ROUNDS=${ROUNDS:-4} timeout -k 10 240 python -u tools/dbg_pose_interference.py \
      > "$out/conc_$v.log" 2>&1
  grep concurrent "$out/conc_$v.log" | tee -a "$out/summary.log"
done
