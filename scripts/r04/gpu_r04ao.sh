#!/bin/bash
# r04ao: the other workloads' bench lines on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04ao
mkdir -p $O
for w in c2 c3 c5 kremling; do
  timeout -k 10 400 python -u bench.py --workload $w > $O/bench_$w.log 2>&1 || { tail -5 $O/bench_$w.log; exit 1; }
  tail -1 $O/bench_$w.log | cut -c1-220
done
