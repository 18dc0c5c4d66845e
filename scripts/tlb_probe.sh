#!/bin/bash
# Which address-translation counters this gfx950 exposes, and their values for the C4
# pass at 64- and 58-row tiles (the 58-row pass is 10 % slower: is it translation?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-tlb}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -i -E "utcl|tlb|translat|TA_BUSY|TCP_TOTAL_CACHE|TCP_PENDING" $O/avail.txt | head -40
for rows in 64 58; do
  for grp in TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum,TCP_UTCL1_PERMISSION_MISS_sum; do
    ROWS=$rows timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $O/p_${rows}_${grp%%,*} -o run -- python3 scripts/stencil_once.py > $O/p_${rows}_${grp%%,*}.log 2>&1 || { echo "pmc $rows $grp failed"; tail -3 $O/p_${rows}_${grp%%,*}.log; break; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
O = 'gpurun_out/' + os.environ.get('TAG', 'tlb')
for f in sorted(glob.glob(O + '/p_*/run_counter_collection.csv')):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'k_diffuse_ps' in r['Kernel_Name']:
            d[r['Counter_Name']].append(float(r['Counter_Value']))
    print(f.split('/')[-2], {k: '%.4g' % (sum(v) / len(v)) for k, v in d.items()})
PY
