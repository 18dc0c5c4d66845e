"""Summarise rocprofv3 --pmc CSVs: per kernel, mean counter value per dispatch."""
import csv, glob, sys, collections
rows = []
for f in sys.argv[1:]:
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r['Kernel_Name'][:48]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print('   %-24s %14.4g  (n=%d)' % (c, sum(v) / len(v), len(v)))
