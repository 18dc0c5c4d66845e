"""C5 rate-law padding by lanes per agent: the padded
rate-law lane-operations one RHS costs when an agent spreads over 64 / 32 / 16 / 8
lanes and each round groups rate laws of similar shape.  CPU only."""
from lens_amd import configs
from lens_amd.rate_law_compiler import compile_rate_laws
from lens_amd.codegen import wave_shape
cfg = configs.synthetic_network(n_species=50, n_reactions=40, n_enzymes=10)
t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
s = wave_shape(t)
num, den = s['num'], s['den']
print('n_params', t.n_params)
def cost(nums, dens):
    # per lane FP64 instr for one rate law slot, padded shape
    SN = max(len(x) for x in nums); MN = max((m for x in nums for m in x), default=0)
    SD = max(len(x) for x in dens)
    md = [max((x[i] if i < len(x) else 0) for x in dens) for i in range(SD)]
    c = SN * (2 * MN) + SN + 1          # num
    c += sum(2 * m for m in md) + 2 * SD   # den
    c += 6                                 # div
    mem = SN * MN + sum(md)
    return c, mem
alg = sum(2*sum(x)+len(x) for x in num) + 40 + sum(2*sum(x)+2*len(x) for x in den) + 6*40
print('algorithmic rate-law lane-ops per RHS', alg)
nl = len(num)
for L in (64, 32, 16, 8):
    R = -(-nl // L)
    # group by den shape: sort by (len sets, members)
    order = sorted(range(nl), key=lambda l: (len(den[l]), sum(den[l]), den[l], sum(num[l])), reverse=True)
    tot = 0; mems = 0
    for r in range(R):
        grp = order[r*L:(r+1)*L]
        c, m = cost([num[l] for l in grp], [den[l] for l in grp])
        tot += c * L; mems += m
    G = 64 // L
    print('lanes/agent %2d rounds %d: padded lane-ops per agent %d (x%.2f), members per lane %d' % (L, R, tot, tot/alg, mems))
