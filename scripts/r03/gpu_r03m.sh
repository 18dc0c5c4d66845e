#!/bin/bash
# Round-3 session m: C4 bench A/B/A/B of the tile rows (64 vs 34) on one box, beside the sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03m
timeout -k 10 200 python -u scripts/stencil_sweep.py 4096 6:9:64:1,6:9:34:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 1; }
cat gpurun_out/${T}_sweep.log
for r in 64 34 64 34; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stencil-rows $r > gpurun_out/bench_${T}_c4_r$r.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4_r$r.log; exit 2; }
  echo "rows $r: $(tail -1 gpurun_out/bench_${T}_c4_r$r.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/bench_${T}_c4_r$r.log | grep -o '"avg_launch_ms": [0-9.]*')"
done
echo session-done
