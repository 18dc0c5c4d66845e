#!/bin/bash
# Round-6 final-tree record: GPU tests, smoke, the driver's bench, its rocprof
# summary, the dominant pass's PMC record (folded into profiles/pmc_stencil_ps_d10.json
# with the commit), the other workloads and a 2-rank gloo rehearsal.  Each GPU step
# has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06final}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
COMMIT=${COMMIT:-unknown}
TAG=$T bash scripts/gpu_session.sh ${STAGES:-tests smoke bench prof} || exit 1
if [ "${PMC:-1}" = 1 ]; then
  i=0
  for grp in FETCH_SIZE WRITE_SIZE \
      SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES,SQ_WAVES,SQ_INSTS_SALU,SQ_WAIT_ANY,GRBM_GUI_ACTIVE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o run -- \
      python3 scripts/stencil_once.py > $O/pmc_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 $O/pmc_$i.log; exit 6; }
  done
  # the bench's own kernel and settings (bench.stencil_settings / stencil_kernel_name at N = 1)
  read KNAME VAR < <(python3 -c "import bench; a = bench.parse([]); m, d, k, r = bench.stencil_settings(a, 1); print(bench.stencil_kernel_name(k, d, m, 16.0 * 4096 * 4096 * 2).replace(' ', '~'), k)")
  KNAME=${KNAME//\~/ }
  python3 scripts/pmc_to_json.py "$KNAME" 33554432 10 64 $VAR \
    $O/pmc_1/run_counter_collection.csv $O/pmc_2/run_counter_collection.csv $O/pmc_stencil_ps_d10.json \
    --sq $O/pmc_3/run_counter_collection.csv --mode fma --commit $COMMIT > $O/pmc_json.log 2>&1 || { cat $O/pmc_json.log; exit 7; }
  tail -1 $O/pmc_json.log | cut -c1-300
fi
if [ "${WORKLOADS_RUN:-1}" = 1 ]; then
  TAG=$T bash scripts/bench_workloads.sh || exit 8
  timeout -k 10 400 python bench.py --stencil-mode exact --no-cpu-baseline --secondary-steps 0 > $O/bench_c4_exact.log 2>&1 || { tail -20 $O/bench_c4_exact.log; exit 9; }
  tail -1 $O/bench_c4_exact.log | cut -c1-200
fi
if [ "${GLOO:-1}" = 1 ]; then
  TAG=$T bash scripts/gpu_session.sh gloo2 || exit 10
fi
echo final-done
