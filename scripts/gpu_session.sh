#!/bin/bash
# A GPU session.  Each argument is a stage, run in order; the session stops at
# the first failure, and every GPU step has its own time limit.
#   tests   pytest -m gpu (every GPU test, one process)
#   smoke   __graft_entry__.smoke()
#   bench   the driver's default bench command (C4 on one GPU)
#   gloo2   bench.py --gpus 2 without a launcher (it starts torch.distributed.run itself;
#           gloo, both ranks on the one GPU)
#   gloo4   the same with 4 ranks
#   prof    rocprofv3 kernel trace + stats of the bench (no counters)
#   pmc     the pass's counters (FETCH_SIZE, WRITE_SIZE, SQ), one rocprofv3 run per group, on
#           scripts/stencil_once.py (DEPTH / ROWS / MODE / VARIANT / REPS from the environment;
#           unset, they default to the C4 bench pass: DEPTH=10 ROWS=64 MODE=fma VARIANT=70)
#   sweep   scripts/stencil_sweep.py with $SWEEP_ARGS
#   cmd     $CMD under a 300 s limit (output in $O/cmd.log)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-session}
mkdir -p $O
export TMPDIR=/tmp
for st in "$@"; do
  case $st in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
      tail -2 $O/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { tail -20 $O/smoke.log; exit 2; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 400 python bench.py > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 3; }
      tail -1 $O/bench_c4.log | cut -c1-400 ;;
    gloo2)
      timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline \
        > $O/bench_gloo2.log 2>&1 || { tail -30 $O/bench_gloo2.log; exit 4; }
      tail -1 $O/bench_gloo2.log | cut -c1-300 ;;
    gloo4)
      timeout -k 10 300 python bench.py --gpus 4 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline \
        > $O/bench_gloo4.log 2>&1 || { tail -30 $O/bench_gloo4.log; exit 4; }
      tail -1 $O/bench_gloo4.log | cut -c1-300 ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
        python3 bench.py --no-cpu-baseline > $O/bench_c4_rocprof.log 2>&1 || { tail -20 $O/bench_c4_rocprof.log; exit 5; }
      tail -1 $O/bench_c4_rocprof.log | cut -c1-300 ;;
    pmc)
      i=0
      for grp in FETCH_SIZE WRITE_SIZE \
          SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES,SQ_WAVES,SQ_INSTS_SALU,SQ_WAIT_ANY,GRBM_GUI_ACTIVE; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o run -- \
          python3 scripts/stencil_once.py > $O/pmc_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 $O/pmc_$i.log; exit 6; }
      done
      echo pmc-done ;;
    sweep)
      timeout -k 10 300 python scripts/stencil_sweep.py $SWEEP_ARGS > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 7; }
      tail -20 $O/sweep.log ;;
    cmd)
      timeout -k 10 300 $CMD > $O/cmd.log 2>&1 || { tail -30 $O/cmd.log; exit 8; }
      tail -30 $O/cmd.log ;;
    *) echo "unknown stage $st"; exit 9 ;;
  esac
done
echo session-done
