#!/bin/bash
# pose build A/B (VARIANTS): parity/accuracy tests per build, timing exact + noisy, bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-default gnsolo}; do
  if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
  echo "== $v"
  MV_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pose.py tests/test_gpu_image_to_pose.py tests/test_gpu_pipeline.py 2>&1 | tail -1
  MV_LIB=$L POSE_BATCHES=8192 POSE_NOISE=1 POSE_HYPS=256 POSE_ITERS=10 timeout -k 10 200 python tools/pose_timing.py 2>&1 | grep "B=" || exit 1
  MV_LIB=$L POSE_BATCHES=8192 POSE_HYPS=256 POSE_ITERS=10 timeout -k 10 200 python tools/pose_timing.py 2>&1 | grep "B=" || exit 1
  MV_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --extra-steps 5 --score-steps 0 --window-steps 0 --no-cpu-baseline --check 1 > gpurun_out/${TAG:-r05ai}_$v.json 2>gpurun_out/${TAG:-r05ai}_$v.err || { tail -5 gpurun_out/${TAG:-r05ai}_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${TAG:-r05ai}_$v.json') if l.startswith('{')][-1])
for k in ('realistic','noisy_pose'):
    v=d.get(k) or {}; print(k, v.get('value'), v.get('stages_ms'), v.get('rot_err_deg'), v.get('tdir_err_deg'), v.get('pose_ok'))
print('headline', d['value'], d['stages_ms_per_step'])"
done
