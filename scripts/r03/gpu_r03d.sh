#!/bin/bash
# Round-3 session d: the whole GPU suite + smoke, every bench workload, the
# Process-API profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r03d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 2; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${T}_c4.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4.log; exit 3; }
tail -1 gpurun_out/bench_${T}_c4.log | cut -c1-200
for w in c3 c2 c5 kremling; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --workload $w > gpurun_out/bench_${T}_$w.log 2>&1 || { tail -20 gpurun_out/bench_${T}_$w.log; exit 4; }
  tail -1 gpurun_out/bench_${T}_$w.log | cut -c1-200
done
timeout -k 10 600 python -u scripts/invoke_profile.py 500 2000 8000 32000 > gpurun_out/${T}_invoke_profile.log 2>&1 || { tail -20 gpurun_out/${T}_invoke_profile.log; exit 5; }
cat gpurun_out/${T}_invoke_profile.log | grep agents
echo session-done
