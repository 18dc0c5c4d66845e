#!/bin/bash
# Round-3 session x: full GPU suite + smoke on the final tree; per-rank diffusion with 10-deep passes
# at N = 2 / 4 / 8 (rank emulation) against 9-deep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03x
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 2; }
tail -1 gpurun_out/${T}_smoke.log
for args in "8 100 16 6 9" "8 100 16 6 10" "8 100 20 6 10" "4 100 0 6 9" "4 100 0 6 10" "2 100 0 6 9" "2 100 0 6 10" "2 100 34 6 10"; do
  timeout -k 10 120 python scripts/rank_emulate.py $args fma >> gpurun_out/${T}_rank_emulate.log 2>&1 || { tail -5 gpurun_out/${T}_rank_emulate.log; exit 3; }
done
grep ms/step gpurun_out/${T}_rank_emulate.log
echo session-done
