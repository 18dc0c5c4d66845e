#!/bin/bash
# Round-3 session t: Process-API loop after the direct kinetics apply (engine GPU tests + min-of-3 timing).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03t
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_registry.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 900 python scripts/invoke_profile.py --profile 32000 500 2000 8000 32000 > gpurun_out/${T}_invoke_profile.log 2>&1 || { tail -10 gpurun_out/${T}_invoke_profile.log; exit 2; }
grep agents gpurun_out/${T}_invoke_profile.log
echo session-done
