"""Where the Process-API path's host time goes (lens_amd.engine.Experiment +
BatchedInvoke + BatchedDiffusionField, scripts/invoke_throughput.py's colony):
per-agent-step cost at several colony sizes, with and without Python's cyclic
GC, and a cProfile of one size.

    python scripts/invoke_profile.py [--profile N] [n_agents ...]

COLUMNS=1 holds the agents in columns (Experiment(config['agent_columns'])).
"""
import cProfile
import gc
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from invoke_throughput import build  # noqa: E402


REPS = int(os.environ.get('INVOKE_REPS', '3'))


def run(n, steps=3, gc_on=True, profile=False):
    from lens_amd.engine import Experiment
    from lens_amd.invoke import BatchedInvoke
    dev = torch.device('cuda', 0)
    p, t, init = build(n, dev)
    cfg = {'processes': p, 'topology': t, 'initial_state': init, 'invoke': BatchedInvoke(dev)}
    if os.environ.get('COLUMNS') == '1':
        cfg['agent_columns'] = ('agents',)
    exp = Experiment(cfg)
    exp.update(1.0)
    torch.cuda.synchronize()
    if not gc_on:
        gc.disable()
    prof = cProfile.Profile() if profile else None
    best = float('inf')
    for _ in range(1 if prof else REPS):    # min of REPS timed calls: the box's host timing is noisy
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        exp.update(float(steps))
        torch.cuda.synchronize()
        if prof:
            prof.disable()
        best = min(best, time.perf_counter() - t0)
    gc.enable()
    print('agents %6d  gc %-3s  %.2f us per agent-step (min of %d calls of %d steps)%s'
          % (n, 'on' if gc_on else 'off', best / (n * steps) * 1e6, 1 if prof else REPS, steps,
             '  [columns]' if os.environ.get('COLUMNS') == '1' else ''), flush=True)
    if prof:
        s = io.StringIO()
        st = pstats.Stats(prof, stream=s)
        st.sort_stats('tottime').print_stats(25)
        st.sort_stats('cumulative').print_stats(30)
        print(s.getvalue(), flush=True)


def main():
    args = sys.argv[1:]
    prof_n = None
    if '--profile' in args:
        i = args.index('--profile')
        prof_n = int(args[i + 1])
        del args[i:i + 2]
    sizes = [int(x) for x in args] or [500, 2000, 8000, 32000]
    for n in sizes:
        run(n, gc_on=True)
        run(n, gc_on=False)
    if prof_n:
        run(prof_n, profile=True)


if __name__ == '__main__':
    main()
