#!/bin/bash
# Round-3 session f: C5 operand tables in LDS (bit-identity + A/B at 2/3 waves per SIMD).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03f
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "wave_spec_equals or wave_vs_c_oracle or wave_matches_odeint" -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 600 python -u scripts/c5_probe.py > gpurun_out/${T}_c5_probe.log 2>&1 || { tail -20 gpurun_out/${T}_c5_probe.log; exit 2; }
cat gpurun_out/${T}_c5_probe.log
echo session-done
