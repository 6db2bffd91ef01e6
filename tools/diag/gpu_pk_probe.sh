#!/bin/bash
# Round-6 diagnosis, third call: the packed-FP32 probe over 16 instruction forms, alone and beside
# three partner workloads, with the first mismatches' operands.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/${TAG:-r06c}
mkdir -p "$out"
timeout -k 10 500 python -u tools/diag/pk_probe.py > "$out/pk_probe.log" 2>&1
grep -E "^form" "$out/pk_probe.log"
