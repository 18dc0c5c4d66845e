#!/bin/bash
# Round-2 GPU session: full GPU tests, smoke, benches (C4 default, Kremling, C5, C2),
# kernel-trace profile of the default bench.  Every GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 3; }
tail -1 gpurun_out/smoke_$TAG.log
for w in ${WORKLOADS:-c4 kremling c5 c2 c3}; do
  steps=20; [ $w = c5 ] && steps=5; [ $w = kremling ] && steps=5; [ $w = c2 ] && steps=100
  timeout -k 10 400 python bench.py --workload $w --steps $steps --warmup 2 > gpurun_out/bench_${TAG}_$w.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$w.log; exit 4; }
  tail -1 gpurun_out/bench_${TAG}_$w.log | cut -c1-400
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 5; }
echo round-done
