#!/bin/bash
# Rows-per-tile sweep of the 10-deep scaled pass around one wave round (3,040 waves at 103 rows).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03sc
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:10:34:1,6:10:103:1,6:10:100:1,6:10:86:1,6:10:120:1,6:10:137:1,6:10:205:1,6:10:256:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 2; }
cat gpurun_out/${T}_sweep.log
echo session-done
