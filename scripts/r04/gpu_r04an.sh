#!/bin/bash
# r04an: counters of the exact mode's 10-deep pass (k_diffuse_wl<10,3,false>, 34-row tiles) for
# bench.py's roofline.traffic / valu_issue on the exact-mode line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04an
mkdir -p $O
export TMPDIR=/tmp
export VARIANT=20 DEPTH=10 ROWS=34 REPS=2 MODE=exact
i=0
for grp in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES,SQ_WAVES,SQ_INSTS_SALU,SQ_WAIT_ANY,GRBM_GUI_ACTIVE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o run -- python3 scripts/stencil_once.py > $O/pmc_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 $O/pmc_$i.log; exit 6; }
done
echo pmc-done
