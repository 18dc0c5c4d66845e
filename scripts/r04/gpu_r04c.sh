#!/bin/bash
# r04c: headline bench (driver's command) with the pair-sum default + rocprof kernel trace of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_c4_rocprof.log 2>&1 || { tail -20 $O/bench_c4_rocprof.log; exit 2; }
tail -1 $O/bench_c4_rocprof.log | cut -c1-300
