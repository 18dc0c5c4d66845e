#!/bin/bash
# r04f: the coupled passes and the dividing-colony loop, the stencil A/B sweep (stagger,
# cache policy, one plane at a time), then the full GPU suite + smoke + bench + rocprof.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_coupled_gpu.py tests/test_engine_gpu.py > $O/pytest_coupled.log 2>&1 || { tail -40 $O/pytest_coupled.log; exit 6; }
tail -2 $O/pytest_coupled.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 20:10:34:1,23:10:34:1,24:10:34:1,25:10:34:1,26:10:34:1,27:10:34:1,26:10:17:1,26:10:26:1,26:10:51:1,23:10:40:1 > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 5; }
cat $O/sweep.log
timeout -k 10 300 python -u scripts/rank_emulate.py 8 --sweep 100:16:20:10,50:16:20:10,50:24:20:10,20:16:20:10,20:24:20:10,100:24:20:10,100:12:20:10,30:16:20:10 > $O/rank_sweep.log 2>&1 || { tail -20 $O/rank_sweep.log; exit 7; }
cat $O/rank_sweep.log
TAG=r04f bash scripts/gpu_full.sh || exit $?
