#!/bin/bash
# SQ counters of the C5 wavefront DP45 kernel (scripts/c5_spec_once.py, 1M agents), two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-c5pmc}; mkdir -p $O
export TMPDIR=/tmp N=${N:-1000000}
i=0
for grp in SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_WAIT_INST_LDS,SQ_INSTS_LDS,SQ_WAIT_ANY,SQ_WAVES \
    SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_SALU,GRBM_GUI_ACTIVE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o run -- python3 scripts/c5_spec_once.py > $O/pmc_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 $O/pmc_$i.log; exit 6; }
done
O=$O python3 - <<'PY'
import csv, collections, glob, os
O = os.environ.get('O') or 'gpurun_out/' + os.environ.get('TAG', 'c5pmc')
d = collections.defaultdict(float)
for f in sorted(glob.glob(O + '/pmc_*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        if 'wspec' in r['Kernel_Name']:
            d[r['Counter_Name']] += float(r['Counter_Value'])
print({k: '%.4g' % v for k, v in sorted(d.items())})
PY
