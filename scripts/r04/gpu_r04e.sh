#!/bin/bash
# r04e: full GPU suite + smoke + bench + rocprof (gpu_full.sh), then a stagger A/B sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r04e bash scripts/gpu_full.sh || exit $?
O=gpurun_out/r04e
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 20:10:34:1,23:10:34:1,24:10:34:1,25:10:34:1,23:10:40:1,23:10:28:1,20:10:34:1,23:10:34:1,24:10:34:1,25:10:34:1 > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 5; }
cat $O/sweep.log
