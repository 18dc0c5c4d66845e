#!/bin/bash
# Round-3 session q: full GPU suite + smoke on the current tree, the driver's bench lines, the other
# workloads, and the Process-API loop at 500-32k agents.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03q
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 2; }
tail -2 gpurun_out/${T}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}_default.log 2>&1 || { tail -20 gpurun_out/bench_${T}_default.log; exit 3; }
tail -1 gpurun_out/bench_${T}_default.log | cut -c1-250
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${T}_c4.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4.log; exit 4; }
tail -1 gpurun_out/bench_${T}_c4.log | cut -c1-250
for w in c2 c3 kremling; do
  timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_${T}_$w.log 2>&1 || { tail -20 gpurun_out/bench_${T}_$w.log; exit 5; }
  tail -1 gpurun_out/bench_${T}_$w.log | cut -c1-200
done
timeout -k 10 600 python scripts/invoke_profile.py 500 2000 8000 32000 > gpurun_out/${T}_invoke_profile.log 2>&1 || { tail -10 gpurun_out/${T}_invoke_profile.log; exit 6; }
grep agents gpurun_out/${T}_invoke_profile.log
echo session-done
