#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, no traces): HBM traffic of the
# C4 step's kernels (exchange, gather, DP45, stencil) and the Kremling kernel's
# issue/wait profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_r02e_c4_$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_r02e_c4_$i.log 2>&1 || { tail -5 gpurun_out/pmc_r02e_c4_$i.log; exit 6; }
done
for grp in SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAIT_ANY GRBM_GUI_ACTIVE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_r02e_krem_$i -o run -- python3 bench.py --workload kremling --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_r02e_krem_$i.log 2>&1 || { tail -5 gpurun_out/pmc_r02e_krem_$i.log; exit 7; }
done
echo pmc-done
