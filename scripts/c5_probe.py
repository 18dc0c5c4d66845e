"""Time the agent-per-wavefront DP45 on the C5 network (50 species, 40 reactions):
the table walk (variant 1) against the specialised kernel (variant 3), with and
without branch-free LDS publishes (KineticsEngine.WAVE_PAD_WRITES) and LDS operand
tables (WAVE_LDS_OPS), and split denominators (WAVE_SPLIT_DEN) at 2 and 3 waves per SIMD.

    python scripts/c5_probe.py [n_agents]
"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from lens_amd import configs
from lens_amd.kinetics import KineticsEngine
from lens_amd.rate_law_compiler import compile_rate_laws
dev = torch.device('cuda', 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
cfg = configs.synthetic_network(n_species=50, n_reactions=40, n_enzymes=10)
t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
print('ny', t.n_dyn + t.n_reactions, 'rate laws', t.n_rate_laws, 'F_rhs', t.flops_rhs(), flush=True)
params, conc = configs.heterogeneous_colony(t, cfg, n, sigma=0.2)
P = torch.from_numpy(params).to(dev)
m2c = torch.full((n,), 7e5, dtype=torch.float64, device=dev)
cases = [('generic', 1, None, 1, 0, 0), ('spec-3w-split', 3, 3, 1, 0, 1), ('spec-3w-split-lds1', 3, 3, 1, 1, 1),
         ('spec-3w-split-lds2', 3, 3, 1, 2, 1), ('spec-4w-split-lds1', 3, 4, 1, 1, 1),
         ('spec-4w-split-lds2', 3, 4, 1, 2, 1)]
if len(sys.argv) > 2 and sys.argv[2] == 'all':
    cases += [('spec-2w', 3, 2, 1, 0, 0), ('spec-2w-split', 3, 2, 1, 0, 1), ('spec-3w-split-nopad', 3, 3, 0, 0, 1)]
first = None
for label, variant, wpe, pad, lds, split in cases + cases[1:]:      # A/B/A/B in one process
    eng = KineticsEngine(t, dev)
    if wpe:
        eng.WAVE_WAVES_PER_SIMD = wpe
        eng.WAVE_PAD_WRITES = pad
        eng.WAVE_LDS_OPS = lds
        eng.WAVE_SPLIT_DEN = split
        eng.specialize()
    C = torch.from_numpy(conc).to(dev)
    h = torch.zeros(n, dtype=torch.float64, device=dev)
    eng.dopri5(1.0, P, C, m2c, h_state=h, variant=variant)          # warm: h carried over
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    flux, counts, st, ns = eng.dopri5(1.0, P, C, m2c, h_state=h, variant=variant)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    nst = ns.double().mean().item()
    fl = ns.double().sum().item() * eng.dopri5_flops_per_attempt()
    same = ''
    if variant == 3:   # every specialised layout computes the table walk's sums: bit-identical outputs
        out = (C.clone(), counts.clone(), ns.clone())
        if first is None:
            first = out
        same = ' bit-identical %s' % all(torch.equal(x, y) for x, y in zip(out, first))
    print('%-8s ms %.2f  attempts/agent %.2f  TF %.2f  agent-steps/s %.3g  status %d%s'
          % (label, dt * 1e3, nst, fl / dt / 1e12, n / dt, int(st.max()), same), flush=True)
