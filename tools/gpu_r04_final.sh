#!/bin/bash
# round 4, the shipping build's record: the whole GPU suite, smoke(), the default bench command,
# then rocprofv3 over the headline (kernel trace + FETCH_SIZE / WRITE_SIZE passes).  STAGE=tests|bench|prof
# runs one part (each part fits one gpurun call).  A failed step ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r04f}
case "${STAGE:-tests}" in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log; exit $rc ;;
bench)
  timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_$TAG.json; exit $rc ;;
prof)
  bash tools/profile.sh $TAG ;;
esac
