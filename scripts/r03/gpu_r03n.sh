#!/bin/bash
# Round-3 session n: final pass with cache-allocating stores (VK_STENCIL_FINAL_TEMPORAL) A/B in the
# C4 bench and under a kernel trace (exchange / gather / final pass); SQ counters of the C5 wave kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03n
for tf in 0 1 0 1; do
  VK_STENCIL_FINAL_TEMPORAL=$tf timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${T}_tf$tf.log 2>&1 || { tail -20 gpurun_out/bench_${T}_tf$tf.log; exit 1; }
  echo "final_temporal $tf: $(tail -1 gpurun_out/bench_${T}_tf$tf.log | grep -o '"ms_per_step": [0-9.]*')"
done
for tf in 0 1; do
  export VK_STENCIL_FINAL_TEMPORAL=$tf
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}_tf$tf -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${T}_tf$tf.log 2>&1 || { tail -20 gpurun_out/prof_${T}_tf$tf.log; exit 2; }
done
unset VK_STENCIL_FINAL_TEMPORAL
python3 scripts/step_kernel_sum.py gpurun_out/prof_${T}_tf0/run_kernel_trace.csv > gpurun_out/${T}_sum_tf0.json
python3 scripts/step_kernel_sum.py gpurun_out/prof_${T}_tf1/run_kernel_trace.csv > gpurun_out/${T}_sum_tf1.json
grep -A9 per_kernel gpurun_out/${T}_sum_tf0.json; grep -A9 per_kernel gpurun_out/${T}_sum_tf1.json
export N=200000
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_${T}_c5 -o run -- python3 scripts/c5_spec_once.py > gpurun_out/pmc_${T}_c5.log 2>&1 || { echo "c5 pmc failed"; tail -5 gpurun_out/pmc_${T}_c5.log; exit 3; }
echo session-done
