#!/bin/bash
# r04g: coupled passes in both modes, the full GPU suite + smoke + bench + rocprof
# (gpu_full.sh), then the other workloads' benches and the exact-mode C4 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_coupled_gpu.py tests/test_gpu_parity.py -k "coupled or banded" > $O/pytest_coupled.log 2>&1 || { tail -40 $O/pytest_coupled.log; exit 6; }
tail -2 $O/pytest_coupled.log
TAG=r04g bash scripts/gpu_full.sh || exit $?
for w in c2 c3 c5 kremling; do
  timeout -k 10 300 python bench.py --workload $w > $O/bench_$w.log 2>&1 || { tail -20 $O/bench_$w.log; exit 8; }
  tail -1 $O/bench_$w.log | cut -c1-250
done
timeout -k 10 300 python bench.py --stencil-mode exact > $O/bench_c4_exact.log 2>&1 || { tail -20 $O/bench_c4_exact.log; exit 9; }
tail -1 $O/bench_c4_exact.log | cut -c1-250
