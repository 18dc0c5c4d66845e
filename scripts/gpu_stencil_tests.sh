#!/bin/bash
# Every stencil-touching GPU test file, one process (after a pass-kernel change).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-stests}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stencil_modes.py tests/test_stencil_split.py tests/test_coupled_gpu.py tests/test_configs.py tests/test_distributed_gpu.py tests/test_graph_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
