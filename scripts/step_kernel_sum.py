"""Per-step kernel time of a bench run from its rocprofv3 kernel trace.

A colony step starts with its kinetics launch (vk_dopri5_spec / _wspec /
k_dopri5_*), so the dispatches between two consecutive kinetics launches are
one step.  For every such step this sums the kernel durations (the GPU work
of the step), and the wall span from the step's first kernel start to the
next step's first kernel start.  Steps whose kernel list differs from the
most common one (setup, the bench's stencil-pass / copy-floor timing loops)
are dropped.  Prints the median step and each kernel's share, to set beside
the bench line's ms_per_step and integrator.avg_ms_per_step.

    python scripts/step_kernel_sum.py run_kernel_trace.csv
"""
import csv
import json
import statistics
import sys
from collections import Counter, defaultdict

KIN = ('vk_dopri5_spec', 'vk_dopri5_wspec', 'k_dopri5_thread', 'k_dopri5_wave', 'k_step_euler')


def short(name):
    name = name.replace('void ', '')
    return name.split('(')[0]


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    steps, cur = [], None
    for r in rows:
        k = short(r['Kernel_Name'])
        if any(k.startswith(p) for p in KIN):
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((k, int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    sig = Counter(tuple(k for k, _, _ in s) for s in steps)
    common, n_common = sig.most_common(1)[0]
    full = [s for s in steps if tuple(k for k, _, _ in s) == common]
    kern_ms = [sum(e - b for _, b, e in s) / 1e6 for s in full]
    span_ms = [(full[i + 1][0][1] - full[i][0][1]) / 1e6 for i in range(len(full) - 1)
               if full[i + 1][0][1] > full[i][-1][2]]
    per = defaultdict(list)
    for s in full:
        acc = defaultdict(float)
        for k, b, e in s:
            acc[k] += (e - b) / 1e6
        for k, v in acc.items():
            per[k].append(v)
    out = {'trace': path, 'steps_matched': len(full), 'steps_total': len(steps),
           'kernels_per_step': len(common),
           'median_step_kernel_ms': statistics.median(kern_ms),
           'median_step_span_ms': statistics.median(span_ms) if span_ms else None,
           'per_kernel_median_ms_per_step': {k: statistics.median(v) for k, v in
                                             sorted(per.items(), key=lambda kv: -statistics.median(kv[1]))}}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1])
