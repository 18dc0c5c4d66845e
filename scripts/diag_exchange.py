import sys, os, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
os.chdir(os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
from test_exchange_in_pass import _pair
from test_coupled_gpu import _stencil
dev = torch.device('cuda', 0)
def cmp(a, b, tag):
    (ca, la), (cb, lb) = a, b
    for m in la.molecules:
        x, y = la.owned(m), lb.owned(m)
        d = (x != y).nonzero()
        print(tag, m, 'mismatches', d.shape[0], d[:8].tolist(), flush=True)
for mode in ('exin', 'coupled20', 'coupled70'):
    for cells in (40, 3):
        kern = 20 if mode == 'coupled20' else 70
        with _stencil('fma', 10, kern, 64):
            a, b = _pair(dev, 128, 300, 3000, 1500, crowd_cells=cells)
            if mode != 'exin':
                a[0].exchange_in_pass = False
                a[0].fuse_coupling = True
            a[0].step(1.0); b[0].step(1.0); torch.cuda.synchronize()
            cmp(a, b, (mode, cells))
