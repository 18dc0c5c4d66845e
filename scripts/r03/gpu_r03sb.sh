#!/bin/bash
# Scaled tolerance-mode stencil: rocprofv3 kernel trace of the driver's command, PMC passes of the
# 10-deep 34-row pass, a rows-per-tile sweep at depth 10.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03sb
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_${T}.log 2>&1 || { tail -20 gpurun_out/prof_${T}.log; exit 3; }
tail -1 gpurun_out/prof_${T}.log | cut -c1-200
export VARIANT=6 DEPTH=10 ROWS=34 REPS=2 MODE=fma
i=0
for grp in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,GRBM_GUI_ACTIVE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- python3 scripts/stencil_once.py > gpurun_out/pmc_${T}_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 gpurun_out/pmc_${T}_$i.log; exit 6; }
done
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 6:10:34:1,6:10:28:1,6:10:40:1,6:10:48:1,6:10:64:1,6:9:34:1 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 2; }
cat gpurun_out/${T}_sweep.log
echo session-done
