#!/bin/bash
# A/B of bench.py argument sets on one box, interleaved rounds:
#     bench_ab.sh 'ARGS_A' 'ARGS_B' [...]     (ROUNDS, default 3; TAG names gpurun_out/TAG)
# e.g. bench_ab.sh '' '--stencil-rows 64'  or  bench_ab.sh '--workload c3' '--workload c3 --stencil-depth 9'.
# Prints ms per step and the dominant pass's roofline fraction for every run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-benchab}; mkdir -p $O
for r in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for args in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --no-cpu-baseline --secondary-steps 0 --steps 20 $args > $O/arm${i}_$r.json 2> $O/arm${i}_$r.err \
      || { echo "arm $i ($args) failed"; tail -5 $O/arm${i}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/arm${i}_$r.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('arm $i [$args] round $r: %.4f ms/step  pass frac %s' % (d['ms_per_step'], r.get('frac')))"
  done
done
