#!/bin/bash
# Exact-mode 10-deep plan: parity suite, then exact C4 at depth 9 / 10 alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_stencil_modes.py tests/test_distributed_gpu.py tests/test_coupled_gpu.py tests/test_configs.py tests/test_graph_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for d in 9 10; do
    timeout -k 10 200 python -u bench.py --stencil-mode exact --stencil-depth $d --no-cpu-baseline > $O/exact_d${d}_$r.log 2>&1 || exit 2
  done
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/fma_c4.log 2>&1 || exit 3
echo done
