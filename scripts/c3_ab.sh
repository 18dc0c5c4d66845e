#!/bin/bash
# C3 pass-plan A/B (one box, interleaved rounds): the default 9-deep variant-20 plan
# against 10-deep passes with variant 20 and with the stage-split variant 40.
# Each bench run is one JSON line; the summary prints ms_per_step per arm.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-c3ab}
mkdir -p $O
run() {  # name, extra args
  timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --steps 40 --warmup 5 "${@:2}" \
    > $O/$1.json 2> $O/$1.err || { echo "arm $1 failed"; tail -5 $O/$1.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('%-14s %.4f ms/step  %.3e' % ('$1', d['ms_per_step'], d['value']))"
}
for r in 1 2; do
  run d9_v20_$r
  run d10_v20_$r --stencil-depth 10
  run d10_v40_$r --stencil-depth 10 --stencil-kernel 40
  run d10_v40r48_$r --stencil-depth 10 --stencil-kernel 40 --stencil-rows 48
  run d10_v40r128_$r --stencil-depth 10 --stencil-kernel 40 --stencil-rows 128
done
echo c3ab-done
