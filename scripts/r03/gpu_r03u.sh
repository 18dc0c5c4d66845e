#!/bin/bash
# Round-3 session u: stencil variant 15 (zigzag chunks) parity + A/B (sweep and whole bench).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03u
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_stencil_modes.py -k "stencil or fma_mode" -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:9:34:1,15:9:34:1,6:9:64:1,15:9:64:1,15:9:52:1,15:9:40:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 2; }
cat gpurun_out/${T}_sweep.log
for k in 6 15 6 15; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stencil-kernel $k > gpurun_out/bench_${T}_k$k.log 2>&1 || { tail -20 gpurun_out/bench_${T}_k$k.log; exit 3; }
  echo "kernel $k: $(tail -1 gpurun_out/bench_${T}_k$k.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/bench_${T}_k$k.log | grep -o '"avg_launch_ms": [0-9.]*')"
done
export VARIANT=15 DEPTH=9 ROWS=34 REPS=2 MODE=fma
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${T}_1 -o run -- python3 scripts/stencil_once.py > gpurun_out/pmc_${T}_1.log 2>&1 || { echo "pmc failed"; exit 4; }
echo session-done
