#!/bin/bash
# Round-3 session h: C5 split denominators (parity + A/B), stencil tile-rows sweep (wave rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03h
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "wave" -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 600 python -u scripts/c5_probe.py > gpurun_out/${T}_c5_probe.log 2>&1 || { tail -20 gpurun_out/${T}_c5_probe.log; exit 2; }
cat gpurun_out/${T}_c5_probe.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:9:64:1,6:9:56:1,6:9:52:1,6:9:48:1,6:9:44:1,6:9:40:1,6:9:34:1,13:9:52:1,13:9:34:1,13:9:24:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 3; }
cat gpurun_out/${T}_sweep.log
echo session-done
