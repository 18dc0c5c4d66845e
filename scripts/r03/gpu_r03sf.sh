#!/bin/bash
# Scaled-form edge tests; variant 16 (10-deep fma pass with 6 rows prefetched, 2 waves/SIMD) A/B sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03sf
timeout -k 10 300 python -u -m pytest tests/test_stencil_modes.py -x -q --timeout 120 --timeout-method thread -k "scaled or zero" > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:10:34:1,16:10:34:1,16:10:52:1,16:10:78:1,16:10:40:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 2; }
cat gpurun_out/${T}_sweep.log
echo session-done
