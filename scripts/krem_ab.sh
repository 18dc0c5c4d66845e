#!/bin/bash
# A/B of two library builds (lens_amd/lib/ab_<arm>.so) on the Kremling workload and its GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-kremab}; mkdir -p $O
for arm in ${ARMS:-k2 k1}; do
  cp lens_amd/lib/ab_$arm.so lens_amd/lib/libvk_kinetics.so
  timeout -k 10 300 python -u -m pytest tests/test_kremling.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$arm.log 2>&1 || { tail -20 $O/pytest_$arm.log; exit 1; }
  echo "$arm tests: $(tail -1 $O/pytest_$arm.log)"
done
for r in 1 2; do
  for arm in ${ARMS:-k2 k1}; do
    cp lens_amd/lib/ab_$arm.so lens_amd/lib/libvk_kinetics.so
    timeout -k 10 300 python bench.py --workload kremling --no-cpu-baseline --steps 10 > $O/${arm}_$r.log 2>&1 || { tail -20 $O/${arm}_$r.log; exit 2; }
    tail -1 $O/${arm}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); i=d.get('integrator') or {}; print('$arm round $r', '%.3e' % d['value'], '%.4f ms' % d['ms_per_step'], 'fp64', i.get('frac'), 'attempts', i.get('dp45_attempts_per_agent_step'))"
  done
done
echo krem-done
