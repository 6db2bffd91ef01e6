#!/bin/bash
# the 16x16x64 int8 all-pairs kernel: parity (every int8 test), then an ABAB A/B against round 5's build
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06ff}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_allpairs.py tests/test_gpu_superpoint.py -x -q -k "i8 or int8" --timeout 240 --timeout-method thread > "$out/pytest_i8.log" 2>&1 || { tail -30 "$out/pytest_i8.log"; exit 1; }
tail -2 "$out/pytest_i8.log"
for r in 1 2; do
  for lib in maveric-slam_amd/libmaveric_hip.so build_variants/libmaveric_i8cur.so; do
    MV_LIB=$lib timeout -k 10 300 python -u tools/bench_i8.py --batch 8192 --steps 10 --warmup 2 --check 1 --cpu-seconds 0 > "$out/$(basename $lib .so)_$r.json" 2>&1 || { tail -5 "$out/$(basename $lib .so)_$r.json"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/$(basename $lib .so)_$r.json').read().strip().splitlines()[-1]); print('$(basename $lib .so)', 'round $r', d['value'], d.get('stages_ms'), d.get('mfma_roofline'))"
  done
done
