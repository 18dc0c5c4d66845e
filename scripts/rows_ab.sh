#!/bin/bash
# C4 bench A/B of the pass's tile rows ($ROWS_A vs $ROWS_B, default 34 / 64), interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-rowsab}; mkdir -p $O
for r in 1 2 3; do
  for rows in ${ROWS_A:-34} ${ROWS_B:-64}; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --stencil-rows $rows > $O/c4_r${rows}_$r.json 2> $O/c4_r${rows}_$r.err \
      || { echo "arm $rows failed"; tail -5 $O/c4_r${rows}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/c4_r${rows}_$r.json').read().strip().splitlines()[-1]); print('rows $rows round $r: %.4f ms/step  pass frac %.3f' % (d['ms_per_step'], d['roofline']['frac']))"
  done
done
