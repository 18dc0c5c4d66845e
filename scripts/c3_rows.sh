#!/bin/bash
# C3 stage-split (variant 40, 10-deep) chunk-rows sweep against the default plan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-c3rows}${SUB:+/$SUB}
mkdir -p $O
run() {
  timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --steps 40 --warmup 5 "${@:2}" \
    > $O/$1.json 2> $O/$1.err || { echo "arm $1 failed"; tail -5 $O/$1.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('%-14s %.4f ms/step  %.3e' % ('$1', d['ms_per_step'], d['value']))"
}
for r in 1 2; do
  run d9_v20_$r
  for rows in ${ROWS:-16 24 32 40 48 64}; do
    run v40r${rows}_$r --stencil-depth 10 --stencil-kernel 40 --stencil-rows $rows
  done
done
echo rows-done
