#!/bin/bash
# C5: agents per workgroup of the wavefront DP45 kernel (VK_WAVE_GROUP), after the
# wavefront parity tests at the candidate size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-c5grp}; mkdir -p $O
VK_WAVE_GROUP=${CAND:-1} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -x -q --timeout 300 \
  --timeout-method thread -k "wave or c5" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in ${GROUPS_AB:-4 1 2 4 1 2}; do
  VK_WAVE_GROUP=$g timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps 10 > $O/c5_g$g.log 2>&1 || { tail -20 $O/c5_g$g.log; exit 2; }
  tail -1 $O/c5_g$g.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); i=d.get('integrator') or {}; print('group $g', '%.4e' % d['value'], '%.3f ms' % d['ms_per_step'], 'kin', '%.2f' % i.get('avg_ms_per_step'), 'fp64', i.get('frac'))"
done
