#!/bin/bash
# A/B of the whole library built with -fno-slp-vectorize (build_variants/libmaveric_allnoslp.so)
# against the shipped build: bench.py without the CPU baseline, alternated twice.
set -u
mkdir -p gpurun_out
for i in $(seq ${N_AB:-2}); do
  for v in default allnoslp; do
    if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
    MV_LIB=$L timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r05am_${v}_$i.json 2> gpurun_out/r05am_${v}_$i.err || exit 1
    python3 - gpurun_out/r05am_${v}_$i.json $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
out = [sys.argv[2], "headline %.0f" % d["value"], str(d["stages_ms_per_step"])]
for k in ("realistic", "noisy_pose", "superpoint", "image_to_pose", "keypoints", "window_frontend", "i8_allpairs"):
    v = d.get(k) or {}
    out.append("%s %s %s" % (k, v.get("value"), v.get("stages_ms")))
print(" | ".join(out))
PY
  done
done
