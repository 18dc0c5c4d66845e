#!/bin/bash
# A/B of two builds of the library on one box (VK_KINETICS_LIB), C4 headline leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-libab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_stencil_modes.py tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "stencil or c4 or bitwise or aligned" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for arm in head new; do
    if [ $arm = head ]; then export VK_KINETICS_LIB=$PWD/${OLD_LIB:-lens_amd/lib/ab/libvk_kinetics_head.so}; else unset VK_KINETICS_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --secondary-steps 0 --steps 20 > $O/${arm}_$r.json 2> $O/${arm}_$r.err || { echo "arm $arm failed"; tail -5 $O/${arm}_$r.err; exit 2; }
    python -c "import json; d=json.loads(open('$O/${arm}_$r.json').read().strip().splitlines()[-1]); print('$arm round $r: %.4f ms/step  pass %.1f us frac %.3f' % (d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3, d['roofline']['frac']))"
  done
done
