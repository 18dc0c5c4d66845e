#!/bin/bash
# Round-3 session g: stencil variants 12 (stage 0 on the prefetch ring) and 13 (+ branch-free
# buffer stores): bit-exactness / tolerance tests, then A/B against variant 6 in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03g
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_stencil_modes.py -k "stencil or fma_mode" -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:9:64:1,12:9:64:1,13:9:64:1,6:9:64:0,12:9:64:0,13:9:64:0,13:9:32:1,13:11:64:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 2; }
cat gpurun_out/${T}_sweep.log
for k in 6 13 6 13; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stencil-kernel $k > gpurun_out/bench_${T}_c4_k$k.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4_k$k.log; exit 3; }
  tail -1 gpurun_out/bench_${T}_c4_k$k.log | cut -c1-160
done
echo session-done
