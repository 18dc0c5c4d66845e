#!/bin/bash
# The scaled / unscaled tolerance-mode forms on both sides of the |c4| cut, and coef = 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03se
timeout -k 10 300 python -u -m pytest tests/test_stencil_modes.py -x -v --timeout 120 --timeout-method thread -k "scaled or zero" > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/${T}_pytest.log | tail -12
echo session-done
