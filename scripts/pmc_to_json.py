"""Fold rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) for one stencil kernel into
profiles/pmc_stencil.json, which bench.py reads for roofline.traffic.

    python scripts/pmc_to_json.py KERNEL CELLS DEPTH ROWS VARIANT fetch.csv write.csv [out.json]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a wide
coalesced streaming read (16 B/lane loads, as this kernel issues) -> x2;
WRITE_SIZE is exact for 16 B/lane stores.
"""
import csv
import json
import sys


def mean_counter(path, kernel, counter):
    per = {}
    for r in csv.DictReader(open(path)):
        name = r['Kernel_Name']
        if (name.startswith(kernel) or name.startswith('void ' + kernel)) and r['Counter_Name'] == counter:
            per[r['Dispatch_Id']] = per.get(r['Dispatch_Id'], 0.0) + float(r['Counter_Value'])
    if not per:
        raise SystemExit('no %s samples for %s in %s' % (counter, kernel, path))
    # a bench's first step runs with a still-uniform plane whose waves exit at once
    # (half the traffic): average the full-work dispatches only
    top = max(per.values())
    vals = [v for v in per.values() if v > 0.7 * top]
    return sum(vals) / len(vals), len(vals)


kernel, cells, depth, rows, variant, fcsv, wcsv = sys.argv[1:8]
out = sys.argv[8] if len(sys.argv) > 8 else 'profiles/pmc_stencil.json'
fetch_kib, nf = mean_counter(fcsv, kernel, 'FETCH_SIZE')
write_kib, nw = mean_counter(wcsv, kernel, 'WRITE_SIZE')
rec = {
    'kernel': kernel, 'cells': int(cells), 'depth': int(depth), 'rows': int(rows), 'variant': int(variant),
    'fetch_size_kib': fetch_kib, 'write_size_kib': write_kib, 'dispatches': [nf, nw],
    'read_bytes_per_launch': 2.0 * fetch_kib * 1024.0,
    'write_bytes_per_launch': write_kib * 1024.0,
    'algorithmic_bytes_per_launch': 16.0 * int(cells),
    'correction': 'FETCH_SIZE x2 (gfx950 wide-load undercount), WRITE_SIZE x1',
}
rec['hbm_bytes_per_launch'] = rec['read_bytes_per_launch'] + rec['write_bytes_per_launch']
json.dump(rec, open(out, 'w'), indent=1)
print(json.dumps(rec))
