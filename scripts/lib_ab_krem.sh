#!/bin/bash
# A/B of two library builds (VK_KINETICS_LIB) on the Kremling workload, after its parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-kremab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "kremling" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for arm in head new; do
    if [ $arm = head ]; then export VK_KINETICS_LIB=$PWD/lens_amd/lib/ab/libvk_kinetics_head.so; else unset VK_KINETICS_LIB; fi
    timeout -k 10 300 python bench.py --workload kremling --no-cpu-baseline --steps 10 > $O/k_${arm}_$r.log 2>&1 || { tail -20 $O/k_${arm}_$r.log; exit 2; }
    tail -1 $O/k_${arm}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm $r', '%.4e' % d['value'], '%.3f ms' % d['ms_per_step'])"
  done
done
