#!/bin/bash
# Round-3 session s: full GPU suite + smoke + every workload after the scaled tolerance-mode stencil; N=8/4/2 band emulation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03sd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 2; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}_default.log 2>&1 || { tail -20 gpurun_out/bench_${T}_default.log; exit 3; }
tail -1 gpurun_out/bench_${T}_default.log | cut -c1-220
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${T}_c4.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4.log; exit 4; }
tail -1 gpurun_out/bench_${T}_c4.log | cut -c1-220
for w in c2 c3 c5 kremling; do
  timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_${T}_$w.log 2>&1 || { tail -20 gpurun_out/bench_${T}_$w.log; exit 5; }
  echo "$w: $(tail -1 gpurun_out/bench_${T}_$w.log | grep -o '"value": [0-9.e+]*') $(tail -1 gpurun_out/bench_${T}_$w.log | grep -o '"ms_per_step": [0-9.]*')"
done

for args in "8 100 16 6 10" "4 100 0 6 10" "2 100 0 6 10"; do
  timeout -k 10 120 python scripts/rank_emulate.py $args fma >> gpurun_out/${T}_rank_emulate.log 2>&1 || { tail -5 gpurun_out/${T}_rank_emulate.log; exit 6; }
done
grep ms/step gpurun_out/${T}_rank_emulate.log
echo session-done
