#!/bin/bash
# C5 A/B on one box: the wavefront DP45 template at HEAD against the working tree's
# (VK_DOPRI5_WAVE_TEMPLATE), alternating, after the C5 parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-c5ab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -x -q --timeout 300 --timeout-method thread \
  -k "wave_spec or c5" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export VK_DOPRI5_WAVE_TEMPLATE=$PWD/scripts/ab/wave_spec_old.hip.in; else unset VK_DOPRI5_WAVE_TEMPLATE; fi
    timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps ${STEPS:-10} > $O/c5_${arm}_$r.log 2>&1 || { tail -20 $O/c5_${arm}_$r.log; exit 2; }
    tail -1 $O/c5_${arm}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); i=d.get('integrator') or {}; print('$arm', '$r', '%.4e' % d['value'], '%.3f ms' % d['ms_per_step'], 'fp64', i.get('frac'), 'kin_ms', i.get('ms_per_step', i.get('kernel_ms')))"
  done
done
