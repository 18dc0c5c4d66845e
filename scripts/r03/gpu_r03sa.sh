#!/bin/bash
# Scaled tolerance-mode stencil (4 FP64 ops per cell-substep): stencil parity, C4/C3 bench, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03sa
timeout -k 10 600 python -u -m pytest tests/test_stencil_modes.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "stencil or banded or depth or diffuse or lattice or field" > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}_default.log 2>&1 || { tail -20 gpurun_out/bench_${T}_default.log; exit 3; }
tail -1 gpurun_out/bench_${T}_default.log | cut -c1-220
timeout -k 10 400 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/bench_${T}_c3.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c3.log; exit 4; }
tail -1 gpurun_out/bench_${T}_c3.log | cut -c1-220
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 5; }
echo session-done
