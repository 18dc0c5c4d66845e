#!/bin/bash
# Kernel-trace profile of a short bench run (no PMC counters in this pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${ARGS:---steps 5 --warmup 2 --no-cpu-baseline}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py $ARGS > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 5; }
tail -1 gpurun_out/prof_$TAG.log
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-220
