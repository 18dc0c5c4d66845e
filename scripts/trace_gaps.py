"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace.

    python scripts/trace_gaps.py <kernel_trace.csv> [first_kernel_substring] [n_steps]

Finds the timed steps of a `bench.py --graph off` run (the kernels from the
first dispatch of the step's opening kernel after warmup), prints per step its
span, busy time and the gaps longer than 3 us, with the kernel that waited.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    opener = sys.argv[2] if len(sys.argv) > 2 else 'k_uniform_probe'
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ks = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows]
    starts = [i for i, k in enumerate(ks) if opener in k[2]]
    n_steps = int(sys.argv[3]) if len(sys.argv) > 3 else len(starts)
    # the last n_steps + 1 step openers: timed steps and the eager split step after them
    starts = starts[-(n_steps + 1):] + [len(ks)]
    for s in range(len(starts) - 1):
        seg = ks[starts[s]:starts[s + 1]]
        # stop the segment at the first kernel that is not part of a colony step
        span = (seg[-1][1] - seg[0][0]) / 1e3
        busy = sum(e - b for b, e, _ in seg) / 1e3
        gaps = []
        for a, b in zip(seg, seg[1:]):
            g = (b[0] - a[1]) / 1e3
            if g > 3.0:
                gaps.append('%.1f us before %s' % (g, b[2][:40]))
        prev_gap = (seg[0][0] - ks[starts[s] - 1][1]) / 1e3 if starts[s] > 0 else 0.0
        print('step %2d: %3d kernels, span %8.1f us, busy %8.1f us, gap before %7.1f us; %s'
              % (s, len(seg), span, busy, prev_gap, '; '.join(gaps[:6])))


if __name__ == '__main__':
    main()
