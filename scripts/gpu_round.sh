#!/bin/bash
# One GPU session: GPU tests, smoke, bench, kernel-trace profile of the bench,
# stencil PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs).  Every step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
STEPS=${STEPS:-10}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 4; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 5; }
export VARIANT=${VARIANT:-6} DEPTH=${DEPTH:-9} ROWS=${ROWS:-64} REPS=2
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${TAG}_$c -o run -- python3 scripts/stencil_once.py > gpurun_out/pmc_${TAG}_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_${TAG}_$c.log; exit 6; }
done
echo round-done
