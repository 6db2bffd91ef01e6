#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05k}
for cfg in "3 1 8" "3 0 10" "4 0 10" "3 0 10"; do
  set -- $cfg
  NP=$1 SYNC=$2 ROUNDS=$3 timeout -k 10 200 python tools/dbg_pipelines.py > gpurun_out/${TAG}_dbg_$1_$2.log 2>&1 || { tail -5 gpurun_out/${TAG}_dbg_$1_$2.log; exit 1; }
  echo "== NP=$1 SYNC=$2 ROUNDS=$3"; grep -v amdgpu.ids gpurun_out/${TAG}_dbg_$1_$2.log | head -20
done
