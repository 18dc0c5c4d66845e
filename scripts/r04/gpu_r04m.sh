#!/bin/bash
# r04m: gloo rehearsals of the multi-rank bench paths on one GPU (C4 row bands at 2 / 4
# ranks, C2 / C5 agent shards at 2), and a cProfile of the Process-API loop at 32k agents.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
P=29611
for spec in "c4 2" "c4 4" "c2 2" "c5 2"; do
  set -- $spec
  P=$((P+1))
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $2 --master-addr 127.0.0.1 --master-port $P bench.py --workload $1 --gpus $2 --steps 5 --warmup 2 --dist-backend gloo --no-cpu-baseline > $O/$1_$2r.log 2>&1 || { tail -30 $O/$1_$2r.log; exit 1; }
  echo "$1 x$2: $(tail -1 $O/$1_$2r.log | cut -c1-200)"
done
timeout -k 10 400 python -u scripts/invoke_profile.py --profile 32000 32000 > $O/invoke_profile_32k.log 2>&1 || { tail -20 $O/invoke_profile_32k.log; exit 2; }
head -60 $O/invoke_profile_32k.log
