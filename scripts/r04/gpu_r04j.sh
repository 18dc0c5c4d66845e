#!/bin/bash
# r04j: the round's record -- full GPU suite + smoke + bench + rocprof (gpu_full.sh), the
# other workloads, the exact-mode C4 bench, row-band rank emulation, Process-API profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04j
mkdir -p $O
TAG=r04j bash scripts/gpu_full.sh || exit $?
for w in c2 c3 c5 kremling; do
  timeout -k 10 300 python bench.py --workload $w > $O/bench_$w.log 2>&1 || { tail -20 $O/bench_$w.log; exit 8; }
  tail -1 $O/bench_$w.log | cut -c1-200
done
timeout -k 10 300 python bench.py --stencil-mode exact > $O/bench_c4_exact.log 2>&1 || { tail -20 $O/bench_c4_exact.log; exit 9; }
tail -1 $O/bench_c4_exact.log | cut -c1-200
for n in 8 4 2; do
  timeout -k 10 300 python -u scripts/rank_emulate.py $n --sweep 100:16:20:10,100:24:20:10,100:34:20:10 > $O/rank_$n.log 2>&1 || { tail -20 $O/rank_$n.log; exit 10; }
  cat $O/rank_$n.log
done
timeout -k 10 600 python -u scripts/invoke_profile.py 500 2000 8000 32000 > $O/invoke_profile.log 2>&1 || { tail -20 $O/invoke_profile.log; exit 11; }
cat $O/invoke_profile.log
