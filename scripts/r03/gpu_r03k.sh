#!/bin/bash
# Round-3 session k: full GPU suite (split denominators default for C5-size networks; stencil
# variants 12-14), C5 probe + bench, stencil A/B sweep (variants x tile rows).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:9:64:1,14:9:64:1,13:9:64:1,6:9:34:1,14:9:34:1,13:9:34:1,6:9:36:1,6:9:32:1,14:9:17:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 4; }
cat gpurun_out/${T}_sweep.log
timeout -k 10 600 python -u scripts/c5_probe.py > gpurun_out/${T}_c5_probe.log 2>&1 || { tail -20 gpurun_out/${T}_c5_probe.log; exit 2; }
cat gpurun_out/${T}_c5_probe.log
timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/bench_${T}_c5.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c5.log; exit 3; }
tail -1 gpurun_out/bench_${T}_c5.log | cut -c1-300
echo session-done
