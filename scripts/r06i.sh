#!/bin/bash
# Round-6 session i: the vertical-stash pass (variants 60-62): its parity tests, a
# variant A/B on the C4 bench (interleaved rounds), FETCH_SIZE of variant 60's pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06i}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stencil_stash.py -x -q --timeout 120 --timeout-method thread > $O/pytest_stash.log 2>&1 || { tail -30 $O/pytest_stash.log; exit 1; }
tail -1 $O/pytest_stash.log
for r in 1 2 3; do
  for v in ${VARIANTS:-20 60 61 62}; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --secondary-steps 0 --steps 20 --stencil-kernel $v > $O/v${v}_$r.json 2> $O/v${v}_$r.err \
      || { echo "variant $v failed"; tail -5 $O/v${v}_$r.err; exit 2; }
    python -c "import json; d=json.loads(open('$O/v${v}_$r.json').read().strip().splitlines()[-1]); print('v$v round $r: %.4f ms/step  pass %.1f us frac %.3f' % (d['ms_per_step'], d['roofline'].get('pass_us', float('nan')), d['roofline']['frac']))"
  done
done
for v in 60; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${grp}_$v -o run -- \
      python3 scripts/stencil_once.py > $O/pmc_${grp}_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/pmc_${grp}_$v.log; exit 3; }
  done
done
echo session-done
