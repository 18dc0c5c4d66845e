"""Time the agent-per-wavefront DP45 on the C5 network (50 species, 40 reactions)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from lens_amd import configs
from lens_amd.kinetics import KineticsEngine
from lens_amd.rate_law_compiler import compile_rate_laws
dev = torch.device('cuda', 0)
cfg = configs.synthetic_network(n_species=50, n_reactions=40, n_enzymes=10)
t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
print('ny', t.n_dyn + t.n_reactions, 'rate laws', t.n_rate_laws, 'F_rhs', t.flops_rhs())
for n in (100_000, 1_000_000):
    params, conc = configs.heterogeneous_colony(t, cfg, n, sigma=0.2)
    eng = KineticsEngine(t, dev)
    P = torch.from_numpy(params).to(dev); C = torch.from_numpy(conc).to(dev)
    m2c = torch.full((n,), 7e5, dtype=torch.float64, device=dev)
    h = torch.zeros(n, dtype=torch.float64, device=dev)
    flux, counts, st, ns = eng.dopri5(1.0, P, C, m2c, h_state=h)
    torch.cuda.synchronize()
    for rep in range(2):
        t0 = time.perf_counter()
        flux, counts, st, ns = eng.dopri5(1.0, P, C, m2c, h_state=h)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    nst = ns.double().mean().item()
    fl = ns.double().sum().item() * eng.dopri5_flops_per_attempt()
    print(n, 'ms %.2f' % (dt * 1e3), 'attempts/agent %.2f' % nst, 'TF %.2f' % (fl / dt / 1e12),
          'agent-steps/s %.3g' % (n / dt), 'status', int(st.max()))
