#!/bin/bash
# A/B of bench.py argument sets on one box, interleaved rounds.  ARMS: "label:args|label:args|..."
# (C4 headline leg only); ROUNDS (default 3); PRE: a command run first (e.g. a parity check).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-arms}; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$PRE" ]; then timeout -k 10 300 bash -c "$PRE" > $O/pre.log 2>&1 || { tail -30 $O/pre.log; exit 1; }; tail -3 $O/pre.log; fi
IFS='|' read -ra A <<< "$ARMS"
for r in $(seq 1 ${ROUNDS:-3}); do
  for arm in "${A[@]}"; do
    lab=${arm%%:*}; args=${arm#*:}
    timeout -k 10 200 python bench.py --no-cpu-baseline --secondary-steps 0 --steps 20 $args > $O/${lab}_$r.json 2> $O/${lab}_$r.err \
      || { echo "arm $lab failed"; tail -5 $O/${lab}_$r.err; exit 2; }
    python -c "import json; d=json.loads(open('$O/${lab}_$r.json').read().strip().splitlines()[-1]); print('$lab round $r: %.4f ms/step  pass %.1f us frac %.3f' % (d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3, d['roofline']['frac']))"
  done
done
echo arms-done
