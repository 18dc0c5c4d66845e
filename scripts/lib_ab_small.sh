#!/bin/bash
# A/B of two library builds (lens_amd/lib/ab_base.so, ab_new.so) on the small
# workloads (C2, C3 benches), interleaved rounds; the new build is left installed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-libabsmall}; mkdir -p $O
for r in 1 2 3; do
  for arm in ${ARMS:-base new}; do
    cp lens_amd/lib/ab_$arm.so lens_amd/lib/libvk_kinetics.so
    line="$arm round $r:"
    for w in c2 c3; do
      timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > $O/${w}_${arm}_$r.json 2> $O/${w}_${arm}_$r.err \
        || { echo "arm $arm $w failed"; tail -5 $O/${w}_${arm}_$r.err; exit 1; }
      line="$line $w $(python -c "import json; d=json.loads(open('$O/${w}_${arm}_$r.json').read().strip().splitlines()[-1]); print('%.3e (%.5f ms)' % (d['value'], d['ms_per_step']))")"
    done
    echo "$line"
  done
done
