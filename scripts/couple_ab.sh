#!/bin/bash
# C4 bench A/B: separate gather / exchange launches (default) against the coupled
# passes (--couple: gather in the first pass, exchange in the last), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-coupleab}; mkdir -p $O
for r in 1 2 3; do
  for arm in plain couple; do
    extra=""; [ $arm = couple ] && extra="--couple"
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 $extra > $O/c4_${arm}_$r.json 2> $O/c4_${arm}_$r.err \
      || { echo "arm $arm failed"; tail -5 $O/c4_${arm}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/c4_${arm}_$r.json').read().strip().splitlines()[-1]); print('$arm round $r: %.4f ms/step' % d['ms_per_step'])"
  done
done
