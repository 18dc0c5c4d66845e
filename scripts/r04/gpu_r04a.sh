#!/bin/bash
# r04a: pair-sum tolerance-mode stencil (variants 20-22) -- parity first, then the
# A/B sweep against variant 6 on the C4 planes, then the new full-size tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
O=gpurun_out/r04a
timeout -k 10 600 python -u -m pytest tests/test_stencil_modes.py -x -q --timeout 120 --timeout-method thread > $O/stencil_modes.log 2>&1 || { tail -30 $O/stencil_modes.log; exit 1; }
tail -2 $O/stencil_modes.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "stencil or uniform or diffuse" --timeout 120 --timeout-method thread > $O/parity_stencil.log 2>&1 || { tail -30 $O/parity_stencil.log; exit 2; }
tail -2 $O/parity_stencil.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:10:34:1,20:10:34:1,21:10:34:1,22:10:34:1,6:9:34:1,20:9:34:1,21:9:34:1,22:9:34:1,20:10:28:1,20:10:40:1,20:10:48:1,20:10:64:1,20:9:64:1 > $O/sweep.log 2>&1 || { tail -30 $O/sweep.log; exit 3; }
cat $O/sweep.log
timeout -k 10 900 python -u -m pytest tests/test_configs.py tests/test_distributed_gpu.py -x -q -k "bench_configuration or sorted_colony or banded or c4_full" --timeout 300 --timeout-method thread > $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 4; }
tail -3 $O/configs.log
