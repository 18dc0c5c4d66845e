#!/bin/bash
# C5: waves per SIMD the wavefront DP45 kernel is compiled for (VK_WAVE_WPE), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-c5wpe}; mkdir -p $O
for w in ${WPES:-3 2 4 3 2 4}; do
  VK_WAVE_WPE=$w timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps 10 > $O/c5_w$w.log 2>&1 || { tail -20 $O/c5_w$w.log; exit 2; }
  tail -1 $O/c5_w$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); i=d.get('integrator') or {}; print('wpe $w', '%.4e' % d['value'], '%.3f ms' % d['ms_per_step'], 'kin', '%.2f' % i.get('avg_ms_per_step'), 'fp64', i.get('frac'))"
done
