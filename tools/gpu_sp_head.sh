#!/bin/bash
# SuperPoint heads: k_sp_head (persistent, weight-stationary; default) against k_sp_conv1x1
# (build_variants/libmaveric_sphead0.so): parity tests, frames/s and image -> pose A/B twice, and
# a per-dispatch kernel trace of the SuperPoint bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r05w}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_superpoint.py tests/test_gpu_image_to_pose.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in default sphead0; do
    if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
    MV_LIB=$L timeout -k 10 200 python tools/bench_superpoint.py --batch 64 --steps 10 --check 0 > gpurun_out/${TAG}_sp_${v}_$rep.log 2>&1 || exit $?
    echo "$v rep $rep superpoint: $(tail -1 gpurun_out/${TAG}_sp_${v}_$rep.log | cut -c1-200)"
    MV_LIB=$L timeout -k 10 200 python tools/bench_image_pose.py --pipelines 2 > gpurun_out/${TAG}_ip_${v}_$rep.json 2>gpurun_out/${TAG}_ip.err || exit $?
    echo "$v rep $rep image_pose: $(cut -c1-400 gpurun_out/${TAG}_ip_${v}_$rep.json)"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_spk -o run -- python3 tools/bench_superpoint.py --batch 64 --steps 3 --warmup 1 --check 0 > gpurun_out/${TAG}_spk.log 2>&1 || { echo trace failed; exit 1; }
