#!/bin/bash
# rocprofv3 kernel-trace stats of the non-default bench workloads (one run each,
# no PMC) and SQ counter passes (their own runs) of the integrator kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02d}
for w in c5 kremling c2 c3; do
  steps=10; [ $w = c5 ] && steps=3; [ $w = kremling ] && steps=3
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$w -o run -- python3 bench.py --workload $w --steps $steps --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}_$w.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_$w.log; exit 5; }
  tail -1 gpurun_out/prof_${TAG}_$w.log | cut -c1-200
done
for grp in SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAIT_ANY,SQ_INSTS_LDS,SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_${TAG}_c5_$(echo $grp | cut -c1-8) -o run -- python3 scripts/c5_spec_once.py > gpurun_out/pmc_${TAG}_c5.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_c5.log; exit 6; }
done
echo prof-done
