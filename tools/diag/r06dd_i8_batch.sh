#!/bin/bash
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for b in 2048 4096 8192; do
  timeout -k 10 300 python -u tools/bench_i8.py --batch $b --steps 10 --warmup 2 --check 1 --cpu-seconds 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('batch', $b, d['value'], d['stages_ms'], d['mfma_roofline']['frac'])" || exit 1
done
