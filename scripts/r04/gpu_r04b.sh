#!/bin/bash
# r04b: counters of the pair-sum 10-deep pass (variant 20, 34-row tiles) and a tile-rows sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp
export VARIANT=20 DEPTH=10 ROWS=34 REPS=2 MODE=fma
i=0
for grp in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES,SQ_WAVES,SQ_INSTS_SALU,SQ_WAIT_ANY,GRBM_GUI_ACTIVE TCC_HIT,TCC_MISS; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o run -- python3 scripts/stencil_once.py > $O/pmc_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 $O/pmc_$i.log; exit 6; }
done
echo pmc-done
timeout -k 10 300 python -u scripts/stencil_sweep.py 4096 20:10:34:1,20:10:52:1,20:10:103:1,20:10:26:1,20:9:34:1,20:9:39:1,20:9:26:1,20:9:20:1,21:9:26:1,6:10:34:1 > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 2; }
cat $O/sweep.log
