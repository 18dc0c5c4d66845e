#!/bin/bash
# Round-3 session b: new GPU tests (registry binding, stencil tolerance mode,
# Kremling capture), stencil exact-vs-fma A/B, Process-API profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_registry.py tests/test_engine_gpu.py tests/test_kremling.py tests/test_stencil_modes.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1 || { tail -30 gpurun_out/r03b_pytest.log; exit 1; }
tail -3 gpurun_out/r03b_pytest.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:9:64:0,6:9:64:1,6:11:64:1,6:7:64:1,6:13:64:1,6:9:32:1 > gpurun_out/r03b_sweep.log 2>&1 || { tail -20 gpurun_out/r03b_sweep.log; exit 2; }
cat gpurun_out/r03b_sweep.log
timeout -k 10 600 python -u scripts/invoke_profile.py --profile 8000 500 8000 32000 > gpurun_out/r03b_invoke_profile.log 2>&1 || { tail -20 gpurun_out/r03b_invoke_profile.log; exit 3; }
head -8 gpurun_out/r03b_invoke_profile.log
