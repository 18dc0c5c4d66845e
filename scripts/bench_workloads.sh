#!/bin/bash
# The bench on every BASELINE workload other than the default C4 (one run each,
# with the CPU baseline), one JSON line per workload in $O/bench_<w>.log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-workloads}; mkdir -p $O
for w in ${WORKLOADS:-c2 c3 c5 kremling}; do
  timeout -k 10 400 python bench.py --workload $w > $O/bench_$w.log 2>&1 || { tail -20 $O/bench_$w.log; exit 1; }
  tail -1 $O/bench_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); i=d.get('integrator') or {}; r=d.get('roofline') or {}; print('$w', '%.3e' % d['value'], '%.4f ms' % d['ms_per_step'], 'fp64', i.get('frac'), 'pass', r.get('frac'))"
done
