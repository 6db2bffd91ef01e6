#!/bin/bash
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for b in 64 128 256 512; do
  timeout -k 10 300 python -u tools/bench_superpoint.py --batch $b --steps 10 --warmup 2 --check 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('batch', d['batch'], d['value'], d['stages_ms'], d['mfma_roofline']['frac'], d.get('oracle_exact'))" || exit 1
done
