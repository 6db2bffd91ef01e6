#!/bin/bash
# headline / sequence / near-threshold A/B of the non-temporal frame-1 DMA in k_q8t_match
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06x}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_allpairs.py tests/test_gpu_sequence.py -x -q --timeout 240 --timeout-method thread > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
for r in 1 2; do
  for lib in maveric-slam_amd/libmaveric_hip.so build_variants/libmaveric_hcur.so; do
    n=$(basename $lib .so)
    MV_LIB=$lib timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --check 1 --extra-steps 5 --window-steps 0 --score-steps 0 > "$out/${n}_$r.json" 2> "$out/${n}_$r.err" || { tail -5 "$out/${n}_$r.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$out/${n}_$r.json').read().strip().splitlines()[-1])
print('$n', 'round $r', d['value'], 'k %.4f' % d['roofline']['avg_launch_ms'], 'seq', d['sequence']['value'], d['sequence']['stages_ms']['k_q8t_match'], 'nt', d['near_threshold']['value'], d['near_threshold']['k_q8t_match_ms'])"
  done
done
