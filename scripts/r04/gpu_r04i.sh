#!/bin/bash
# r04i: vector-ring pair-sum variants 30-32 -- stencil-mode tests, then the A/B sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_stencil_modes.py > $O/pytest_stencil.log 2>&1 || { tail -40 $O/pytest_stencil.log; exit 6; }
tail -2 $O/pytest_stencil.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 20:10:34:1,30:10:34:1,31:10:34:1,32:10:34:1,30:10:28:1,30:10:40:1,20:10:34:1,30:10:34:1,31:10:34:1,30:9:34:1 > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 5; }
cat $O/sweep.log
