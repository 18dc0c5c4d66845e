#!/bin/bash
# (Record of a reverted experiment: variant 77 is no longer built; DESIGN §10, profiles/r06/pairs.)
# Variant 77 (paired, half-rotated chunk order) against variant 70: bitwise tests, the
# bench A/B (C4 headline leg), and each kernel's FETCH_SIZE / WRITE_SIZE.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-pairs}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_stencil_modes.py -x -q --timeout 300 --timeout-method thread -k "paired or aligned" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/parity_variant.py 77 > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in 70 77; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${v}_$grp -o run -- python3 scripts/stencil_once.py > $O/pmc_${v}_$grp.log 2>&1 || { echo "pmc $v $grp failed"; exit 6; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
O = 'gpurun_out/' + os.environ.get('TAG', 'pairs')
for v in (70, 77):
    out = {}
    for grp in ('FETCH_SIZE', 'WRITE_SIZE'):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open('%s/pmc_%d_%s/run_counter_collection.csv' % (O, v, grp))):
            if 'k_diffuse_p' in r['Kernel_Name'] and '10, 4, 2' in r['Kernel_Name']:
                vals[r['Dispatch_Id']].append(float(r['Counter_Value']))
        per = [sum(x) for x in vals.values()]
        out[grp] = sum(per) / len(per) / 1024 if per else None
    print('variant', v, 'FETCH MB x2 %.1f' % (2 * out['FETCH_SIZE'] * 1.024 * 1.024 / 1.024) if out['FETCH_SIZE'] else None, 'WRITE MB %.1f' % (out['WRITE_SIZE'] * 1.024 * 1.024 / 1.024) if out['WRITE_SIZE'] else None)
PY
TAG=$TAG ARMS="v70:--stencil-kernel 70|v77:--stencil-kernel 77" ROUNDS=${ROUNDS:-3} bash scripts/bench_arms.sh
