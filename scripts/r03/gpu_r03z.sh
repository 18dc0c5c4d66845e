#!/bin/bash
# Round-3 session z: gloo rehearsals of C4 at 2 / 4 ranks with the 10-deep default; C3 depth A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03z
P=29581
for n in 2 4; do
  P=$((P+1))
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $P bench.py --gpus $n --steps 5 --warmup 2 --dist-backend gloo --no-cpu-baseline > gpurun_out/${T}_c4_${n}r.log 2>&1 || { tail -30 gpurun_out/${T}_c4_${n}r.log; exit 1; }
  echo "c4 x$n: $(tail -1 gpurun_out/${T}_c4_${n}r.log | cut -c1-160)"
done
for d in 9 10 9 10; do
  timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --stencil-depth $d > gpurun_out/bench_${T}_c3_d$d.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c3_d$d.log; exit 2; }
  echo "c3 depth $d: $(tail -1 gpurun_out/bench_${T}_c3_d$d.log | grep -o '"ms_per_step": [0-9.]*')"
done
echo session-done
