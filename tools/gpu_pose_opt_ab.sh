#!/bin/bash
# A/B of the pose library variants in build_variants/: cross-stream determinism beside the
# SuperPoint network and the exact / noisy pose timings (profiles/r05al_pose_noslp_ab.log).
set -u
for v in ${VARIANTS:-default posenoslp}; do
  if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
  echo "== $v: $(MV_LIB=$L STAGES=net ROUNDS=4 timeout -k 10 300 python tools/dbg_pose_interference.py 2>&1 | grep concurrent)"
  MV_LIB=$L POSE_BATCHES=8192 POSE_HYPS=256 POSE_ITERS=10 timeout -k 10 200 python tools/pose_timing.py 2>&1 | grep "B=" || exit 1
  MV_LIB=$L POSE_BATCHES=8192 POSE_NOISE=1 POSE_HYPS=256 POSE_ITERS=10 timeout -k 10 200 python tools/pose_timing.py 2>&1 | grep "B=" || exit 1
done
