#!/bin/bash
# Round-3 session v: tolerance-mode 10-deep whole-step plan (10 passes per 100 substeps) parity + A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03v
timeout -k 10 500 python -u -m pytest tests/test_stencil_modes.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:9:34:1,6:10:34:1,6:10:30:1,6:10:40:1,6:10:64:1,6:9:64:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 2; }
cat gpurun_out/${T}_sweep.log
for d in 9 10 9 10; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stencil-depth $d > gpurun_out/bench_${T}_d$d.log 2>&1 || { tail -20 gpurun_out/bench_${T}_d$d.log; exit 3; }
  echo "depth $d: $(tail -1 gpurun_out/bench_${T}_d$d.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/bench_${T}_d$d.log | grep -o '"avg_launch_ms": [0-9.]*')"
done
echo session-done
