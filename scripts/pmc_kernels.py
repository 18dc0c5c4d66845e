"""Per-kernel means of rocprofv3 --pmc passes (one directory per pass):

    python scripts/pmc_kernels.py gpurun_out/r06f/pmc_1 gpurun_out/r06f/pmc_2 ... [--skip N]

For each kernel name (argument list dropped), the mean of every counter over its
dispatches (the first N dispatches of each kernel skipped) and the mean dispatch
duration.  FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE is also shown x2 (the
gfx950 correction for wide coalesced reads, MI355X_MICROARCH.md HBM section)."""
import collections
import csv
import glob
import os
import sys


def base(name):
    if name.startswith('void '):
        name = name[5:]
    d = 0
    for i, ch in enumerate(name):
        d += ch == '<'
        d -= ch == '>'
        if ch == '(' and d == 0:
            return name[:i]
    return name


def main(argv):
    skip = 0
    if '--skip' in argv:
        i = argv.index('--skip')
        skip = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for d in argv:
        for f in glob.glob(os.path.join(d, '*counter_collection.csv')):
            seen = collections.Counter()
            per = collections.defaultdict(dict)
            for r in csv.DictReader(open(f)):
                k = base(r['Kernel_Name'])
                per[(k, int(r['Dispatch_Id']))][r['Counter_Name']] = float(r['Counter_Value'])
                per[(k, int(r['Dispatch_Id']))]['_ns'] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            for (k, disp), cs in sorted(per.items(), key=lambda x: x[0][1]):
                seen[k] += 1
                if seen[k] <= skip:
                    continue
                for c, v in cs.items():
                    if c == '_ns':
                        durs[k].append(v)
                    else:
                        vals[k][c].append(v)
    for k in sorted(vals, key=lambda k: -sum(durs[k]) / max(1, len(durs[k]))):
        line = ['%-48s' % k[:48], 'us %.1f' % (sum(durs[k]) / len(durs[k]) / 1e3)]
        for c, v in sorted(vals[k].items()):
            m = sum(v) / len(v)
            if c == 'FETCH_SIZE':
                line.append('FETCH %.1f MB (x2 %.1f)' % (m * 1024 / 1e6, 2 * m * 1024 / 1e6))
            elif c == 'WRITE_SIZE':
                line.append('WRITE %.1f MB' % (m * 1024 / 1e6))
            else:
                line.append('%s %.4g' % (c, m))
        print('  '.join(line))


if __name__ == '__main__':
    main(sys.argv[1:])
