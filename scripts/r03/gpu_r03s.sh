#!/bin/bash
# Round-3 session s: per-rank diffusion at N = 8 with deeper passes (fewer launches per step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03s
for args in "8 100 16 6 9" "8 100 16 6 11" "8 100 24 6 11" "8 100 16 6 13" "8 100 24 6 13" "8 100 32 6 13" "8 100 24 6 15" "8 100 16 6 9" "4 100 0 6 9" "4 100 32 6 11" "4 100 48 6 13"; do
  timeout -k 10 120 python scripts/rank_emulate.py $args fma >> gpurun_out/${T}_rank_emulate.log 2>&1 || { tail -5 gpurun_out/${T}_rank_emulate.log; exit 1; }
done
grep ms/step gpurun_out/${T}_rank_emulate.log
echo session-done
