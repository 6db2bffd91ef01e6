#!/bin/bash
# SuperPoint build variants (VARIANTS: names of build_variants/libmaveric_<name>.so; "default" =
# the shipping build): parity tests on each non-default variant's library, then frames/s twice,
# interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05x}
for v in ${VARIANTS}; do
  [ $v = default ] && continue
  MV_LIB=build_variants/libmaveric_$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_superpoint.py > gpurun_out/${TAG}_pytest_$v.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in ${VARIANTS}; do
    if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
    MV_LIB=$L timeout -k 10 200 python tools/bench_superpoint.py --batch 64 --steps 10 --check 0 > gpurun_out/${TAG}_sp_${v}_$rep.log 2>&1 || exit $?
    echo "$v rep $rep: $(tail -1 gpurun_out/${TAG}_sp_${v}_$rep.log | cut -c1-150)"
  done
done
