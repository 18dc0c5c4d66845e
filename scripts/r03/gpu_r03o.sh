#!/bin/bash
# Round-3 session o: per-rank diffusion vs tile rows at N = 8 / 2 (wave rounds), C4 depth-11 plans.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03o
for args in "8 100 16" "8 100 18" "8 100 20" "8 100 16" "8 100 18" "2 100 0" "2 100 27" "2 100 34" "4 100 0" "4 100 24"; do
  timeout -k 10 120 python scripts/rank_emulate.py $args 6 9 fma >> gpurun_out/${T}_rank_emulate.log 2>&1 || { tail -5 gpurun_out/${T}_rank_emulate.log; exit 1; }
done
grep ms/step gpurun_out/${T}_rank_emulate.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:9:34:1,6:11:36:1,6:11:34:1,6:11:40:1,6:11:38:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 2; }
cat gpurun_out/${T}_sweep.log
echo session-done
