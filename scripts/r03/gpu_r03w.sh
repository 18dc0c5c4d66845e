#!/bin/bash
# Round-3 session w: the C4 default with 10-deep passes: bench (defaults and the driver's command),
# rocprofv3 kernel trace of the driver's command, PMC passes of the 10-deep 34-row fma pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03w
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}_default.log 2>&1 || { tail -20 gpurun_out/bench_${T}_default.log; exit 1; }
tail -1 gpurun_out/bench_${T}_default.log | cut -c1-200
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${T}_c4.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4.log; exit 2; }
tail -1 gpurun_out/bench_${T}_c4.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${T}.log 2>&1 || { tail -20 gpurun_out/prof_${T}.log; exit 3; }
export VARIANT=6 DEPTH=10 ROWS=34 REPS=2 MODE=fma
i=0
for grp in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,GRBM_GUI_ACTIVE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- python3 scripts/stencil_once.py > gpurun_out/pmc_${T}_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 gpurun_out/pmc_${T}_$i.log; exit 6; }
done
echo session-done
