#!/bin/bash
# Record of a reverted experiment (profiles/r06/stag): builds with VK_PS_STAGGER
# (first-round waves sleeping 0 / 1 / 2 phases before their fill) against the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/stag; mkdir -p $O
for r in 1 2; do
  for arm in head stag2 stag4; do
    if [ $arm = head ]; then L=libvk_kinetics_head.so; else L=libvk_$arm.so; fi
    VK_KINETICS_LIB=$PWD/lens_amd/lib/ab/$L timeout -k 10 200 python bench.py --no-cpu-baseline --secondary-steps 0 --steps 20 > $O/${arm}_$r.json 2> $O/${arm}_$r.err || { echo "arm $arm failed"; tail -5 $O/${arm}_$r.err; exit 2; }
    python -c "import json; d=json.loads(open('$O/${arm}_$r.json').read().strip().splitlines()[-1]); print('$arm round $r: %.4f ms/step  pass %.1f us' % (d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3))"
  done
done
