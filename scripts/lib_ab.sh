#!/bin/bash
# A/B of builds of the library (lens_amd/lib/ab_<arm>.so for each arm in $ARMS,
# default "base new") on the C4 bench, interleaved rounds; the last arm is left
# installed.  $EXTRA: bench args.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-libab}; mkdir -p $O
for r in 1 2 3; do
  for arm in ${ARMS:-base new}; do
    cp lens_amd/lib/ab_$arm.so lens_amd/lib/libvk_kinetics.so
    timeout -k 10 200 python bench.py --no-cpu-baseline --secondary-steps 0 --steps 20 $EXTRA > $O/${arm}_$r.json 2> $O/${arm}_$r.err \
      || { echo "arm $arm failed"; tail -5 $O/${arm}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/${arm}_$r.json').read().strip().splitlines()[-1]); print('$arm round $r: %.4f ms/step  pass frac %.3f' % (d['ms_per_step'], d['roofline']['frac']))"
  done
done
