#!/bin/bash
# One-Newton-step division in every convenience-kinetics DP45 kernel: the whole GPU
# suite, then C5 against HEAD's wavefront template, then the C4 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-divab}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for arm in new old new old; do
  if [ $arm = old ]; then export VK_DOPRI5_WAVE_TEMPLATE=$PWD/scripts/ab/wave_spec_old.hip.in; else unset VK_DOPRI5_WAVE_TEMPLATE; fi
  timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps 10 > $O/c5_$arm.log 2>&1 || { tail -20 $O/c5_$arm.log; exit 2; }
  tail -1 $O/c5_$arm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); i=d.get('integrator') or {}; print('c5 $arm', '%.4e' % d['value'], '%.3f ms' % d['ms_per_step'], 'fp64', i.get('frac'), 'att', i.get('dp45_attempts_per_agent_step'))"
done
unset VK_DOPRI5_WAVE_TEMPLATE
timeout -k 10 400 python bench.py --no-cpu-baseline --secondary-steps 0 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 3; }
tail -1 $O/c4.log | cut -c1-300
