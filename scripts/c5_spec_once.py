"""Two C5-network DP45 steps with the network-specialised agent-per-wavefront
kernel (variant 3) on N agents (default 100k) -- profiling driver for PMC passes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from lens_amd import configs
from lens_amd.kinetics import KineticsEngine
from lens_amd.rate_law_compiler import compile_rate_laws
dev = torch.device('cuda', 0)
cfg = configs.synthetic_network(n_species=50, n_reactions=40, n_enzymes=10)
t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
n = int(os.environ.get('N', '100000'))
params, conc = configs.heterogeneous_colony(t, cfg, n, sigma=0.2)
eng = KineticsEngine(t, dev)
eng.specialize()
P = torch.from_numpy(params).to(dev); C = torch.from_numpy(conc).to(dev)
m2c = torch.full((n,), 7e5, dtype=torch.float64, device=dev)
h = torch.zeros(n, dtype=torch.float64, device=dev)
for _ in range(2):
    eng.dopri5(1.0, P, C, m2c, h_state=h, variant=3)
torch.cuda.synchronize()
print('done')
