"""Fold rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) for one stencil kernel into
profiles/pmc_stencil.json, which bench.py reads for roofline.traffic.

    python scripts/pmc_to_json.py KERNEL CELLS DEPTH ROWS VARIANT fetch.csv write.csv [out.json] [--sq sq.csv]
                                  [--mode exact|fma] [--commit SHA]

KERNEL is the kernel's full template name as rocprofv3 prints it (e.g.
'vk_ps::k_diffuse_ps<10, 4, 2, true, 0>'); a dispatch matches only if its name,
without a leading 'void ' and its argument list, is exactly that.  --commit
records the tree the counters were taken on (bench.py names it in
roofline.traffic_from, and refuses a record whose kernel differs from the one
it launches).

--sq: a pass with SQ_INSTS_VALU and GRBM_GUI_ACTIVE adds the VALU instructions
per launch and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall), from
which bench.py reports the pass against the VALU-issue bound as well.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a wide
coalesced streaming read (16 B/lane loads, as this kernel issues) -> x2;
WRITE_SIZE is exact for 16 B/lane stores.
"""
import csv
import json
import sys


def base_name(name):
    """'void ns::k<1, 2>(double const*, int)' -> 'ns::k<1, 2>'"""
    if name.startswith('void '):
        name = name[5:]
    depth = 0
    for i, ch in enumerate(name):
        depth += ch == '<'
        depth -= ch == '>'
        if ch == '(' and depth == 0:
            return name[:i].strip()
    return name.strip()


def mean_counter(path, kernel, counter):
    per = {}
    for r in csv.DictReader(open(path)):
        name = r['Kernel_Name']
        if base_name(name) == kernel and r['Counter_Name'] == counter:
            per[r['Dispatch_Id']] = per.get(r['Dispatch_Id'], 0.0) + float(r['Counter_Value'])
    if not per:
        raise SystemExit('no %s samples for %s in %s' % (counter, kernel, path))
    # a bench's first step runs with a still-uniform plane whose waves exit at once
    # (half the traffic): average the full-work dispatches only
    top = max(per.values())
    vals = [v for v in per.values() if v > 0.7 * top]
    return sum(vals) / len(vals), len(vals)


argv = list(sys.argv[1:])
mode = 'exact'
if '--mode' in argv:
    i = argv.index('--mode')
    mode = argv[i + 1]
    del argv[i:i + 2]
commit = None
if '--commit' in argv:
    i = argv.index('--commit')
    commit = argv[i + 1]
    del argv[i:i + 2]
sq = None
if '--sq' in argv:
    i = argv.index('--sq')
    sq = argv[i + 1]
    del argv[i:i + 2]
kernel, cells, depth, rows, variant, fcsv, wcsv = argv[:7]
out = argv[7] if len(argv) > 7 else 'profiles/pmc_stencil.json'
fetch_kib, nf = mean_counter(fcsv, kernel, 'FETCH_SIZE')
write_kib, nw = mean_counter(wcsv, kernel, 'WRITE_SIZE')
rec = {
    'kernel': kernel, 'cells': int(cells), 'depth': int(depth), 'rows': int(rows), 'variant': int(variant),
    'mode': mode, 'commit': commit,
    'fetch_size_kib': fetch_kib, 'write_size_kib': write_kib, 'dispatches': [nf, nw],
    'read_bytes_per_launch': 2.0 * fetch_kib * 1024.0,
    'write_bytes_per_launch': write_kib * 1024.0,
    'algorithmic_bytes_per_launch': 16.0 * int(cells),
    'correction': 'FETCH_SIZE x2 (gfx950 wide-load undercount), WRITE_SIZE x1',
}
rec['hbm_bytes_per_launch'] = rec['read_bytes_per_launch'] + rec['write_bytes_per_launch']
if sq:
    per = {}
    for r in csv.DictReader(open(sq)):
        name = r['Kernel_Name']
        if base_name(name) == kernel:
            d = per.setdefault(r['Dispatch_Id'], {'ns': int(r['End_Timestamp']) - int(r['Start_Timestamp'])})
            d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    top = max(d['SQ_INSTS_VALU'] for d in per.values())
    full = [d for d in per.values() if d['SQ_INSTS_VALU'] > 0.7 * top]
    rec['valu_insts_per_launch'] = sum(d['SQ_INSTS_VALU'] for d in full) / len(full)
    rec['clock_ghz'] = sum(d['GRBM_GUI_ACTIVE'] / 8 / d['ns'] for d in full) / len(full)
    rec['valu_busy_per_simd'] = sum(d['SQ_ACTIVE_INST_VALU'] * 4 / 1024 / (d['GRBM_GUI_ACTIVE'] / 8)
                                    for d in full) / len(full) if 'SQ_ACTIVE_INST_VALU' in full[0] else None
json.dump(rec, open(out, 'w'), indent=1)
print(json.dumps(rec))
