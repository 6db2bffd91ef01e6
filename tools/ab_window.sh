#!/bin/bash
# A/B of library builds on the windowed front-end (tools/bench_window.py at the bench's batch):
# LIBS="a.so b.so", each run ROUNDS times interleaved; prints pairs/s and the per-kernel ms.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-abw}
mkdir -p "$out"
ARGS=${ARGS:-"--batch 8192 --steps 20 --warmup 3 --check 2 --cpu-seconds 0"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS}; do
    n=$(basename $lib .so)
    MV_LIB=$lib timeout -k 10 300 python -u tools/bench_window.py $ARGS > "$out/${n}_$r.json" 2> "$out/${n}_$r.err"
    python3 -c "import json; d=json.loads(open('$out/${n}_$r.json').read().strip().splitlines()[-1]); print('$n', 'round $r', d['value'], d['stages_ms'], 'checked', d['checked_pairs'])" | tee -a "$out/summary.log"
  done
done
