#!/bin/bash
# Round-3 session j: stencil variant 14 (ring + buffer stores, 3-row lookahead) parity + A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03j
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_stencil_modes.py -k "stencil or fma_mode" -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:9:64:1,14:9:64:1,13:9:64:1,6:9:34:1,14:9:34:1,13:9:34:1,14:9:17:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 2; }
cat gpurun_out/${T}_sweep.log
echo session-done
