#!/bin/bash
# Round-3 session r: multi-rank rehearsals on one GPU (gloo, device tensors staged through host) of
# the driver's N > 1 command shapes on the final tree: C4 at 2 and 4 ranks, C5 at 2 ranks, C2 at 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03r
P=29541
for spec in "c4 2" "c4 4" "c5 2" "c2 2"; do
  set -- $spec
  P=$((P+1))
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus $2 --steps 5 --warmup 2 --workload $1 --dist-backend gloo --no-cpu-baseline > gpurun_out/${T}_$1_$2r.log 2>&1 || { tail -30 gpurun_out/${T}_$1_$2r.log; exit 1; }
  echo "$1 x$2: $(tail -1 gpurun_out/${T}_$1_$2r.log | cut -c1-200)"
done
echo session-done
