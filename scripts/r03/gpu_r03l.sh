#!/bin/bash
# Round-3 session l: split-denominator continuation with one select (bit-identity + A/B), C5 bench,
# C4 bench with 34-row tiles (the driver's command), its rocprofv3 kernel trace, PMC passes of the
# 34-row fma pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03l
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -k "wave or c5" -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 600 python -u scripts/c5_probe.py > gpurun_out/${T}_c5_probe.log 2>&1 || { tail -20 gpurun_out/${T}_c5_probe.log; exit 2; }
cat gpurun_out/${T}_c5_probe.log
timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/bench_${T}_c5.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c5.log; exit 3; }
tail -1 gpurun_out/bench_${T}_c5.log | cut -c1-200
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${T}_c4.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4.log; exit 4; }
tail -1 gpurun_out/bench_${T}_c4.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${T}.log 2>&1 || { tail -20 gpurun_out/prof_${T}.log; exit 5; }
export VARIANT=6 DEPTH=9 ROWS=34 REPS=2 MODE=fma
i=0
for grp in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,GRBM_GUI_ACTIVE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- python3 scripts/stencil_once.py > gpurun_out/pmc_${T}_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 gpurun_out/pmc_${T}_$i.log; exit 6; }
done
echo session-done
