"""Rate-law code generator: RateLawTable -> network-specialised HIP source.

The generic kernels walk the flat table at run time (species in an LDS tile,
indices through the scalar cache).  For a fixed network the same arithmetic
can be emitted as straight-line code with every species, parameter and stage
vector in VGPRs at compile-time indices; ``vk_table_specialize`` compiles it
with hiprtc for gfx950 and the ODE step uses it (variant 2).

The emitted rate law is the one the generic DP45 kernel evaluates
(kinetic_rate_laws.py:149-178 with 1/Km precomputed): for each numerator set
``kcat * prod(c*invKm)``, times the enzyme, over ``1 + sum(prod(1 + c*invKm) - 1)``.
"""

from __future__ import annotations

import os

from lens_amd.rate_law_compiler import RateLawTable

TEMPLATE = os.environ.get('VK_DOPRI5_TEMPLATE') or os.path.join(os.path.dirname(os.path.abspath(__file__)), 'csrc',
                                                                 'vk_dopri5_spec.hip.in')


def _f(x: float) -> str:
    return repr(float(x))


def rhs_body(t: RateLawTable) -> str:
    lines = []
    nd = t.n_dyn
    for r in range(t.n_reactions):
        lines.append('    double f%d = 0.0;' % r)
    for l in range(t.n_rate_laws):
        rid, enz = t.rate_laws[l]
        lines.append('    {  // %s / %s' % (rid, enz[1] if isinstance(enz, tuple) else enz))
        lines.append('        double num = 0.0;')
        for s in range(t.rl_num_ptr[l], t.rl_num_ptr[l + 1]):
            terms = ['p[%d]' % t.rl_kcat[l]]
            for m in range(t.set_ptr[s], t.set_ptr[s + 1]):
                terms.append('(c[%d] * p[%d])' % (t.mem_species[m], t.mem_param[m]))
            lines.append('        num += %s;' % ' * '.join(terms))
        lines.append('        num *= c[%d];' % t.rl_enzyme[l])
        lines.append('        double den = 1.0;')
        for s in range(t.rl_den_ptr[l], t.rl_den_ptr[l + 1]):
            terms = ['fma(c[%d], p[%d], 1.0)' % (t.mem_species[m], t.mem_param[m])
                     for m in range(t.set_ptr[s], t.set_ptr[s + 1])]
            lines.append('        den += %s - 1.0;' % (' * '.join(terms) if terms else '1.0'))
        lines.append('        f%d += vk_div(num, den);' % t.rl_reaction[l])
        lines.append('    }')
    for i in range(nd):
        expr = '0.0'
        for j in range(t.upd_ptr[i], t.upd_ptr[i + 1]):
            expr = 'fma(%s, f%d, %s)' % (_f(t.upd_coeff[j]), t.upd_rxn[j], expr)
        lines.append('    dy[%d] = %s;' % (i, expr))
    for r in range(t.n_reactions):
        lines.append('    dy[%d] = f%d;' % (nd + r, r))
    return '\n'.join(lines)


def counts_body(t: RateLawTable) -> str:
    lines = []
    for e in range(t.n_ext):
        lines.append('    {')
        lines.append('        i64 cnt = 0;')
        for j in range(t.ex_ptr[e], t.ex_ptr[e + 1]):
            lines.append('        cnt += trunc_count((%s * y[%d]) * mc, st);'
                         % (_f(t.ex_coeff[j]), t.n_dyn + t.ex_rxn[j]))
        lines.append('        counts[(i64)%d * ld + a] = cnt;' % e)
        lines.append('    }')
    return '\n'.join(lines)


def invkm_body(t: RateLawTable) -> str:
    km_rows = sorted(set(int(x) for x in t.mem_param))
    return '\n'.join('    p[%d] = (p[%d] != 0.0) ? 1.0 / p[%d] : 0.0;' % (q, q, q) for q in km_rows)


def dopri5_source(t: RateLawTable) -> str:
    """Complete HIP source of the specialised ``vk_dopri5_spec`` kernel."""
    with open(TEMPLATE) as f:
        src = f.read()
    defs = '\n'.join([
        '#define NS %d' % max(t.n_species, 1),
        '#define ND %d' % t.n_dyn,
        '#define NR %d' % t.n_reactions,
        '#define NP %d' % max(t.n_params, 1),
        '#define NP_REAL %d' % t.n_params,
        '#define NY %d' % max(t.n_dyn + t.n_reactions, 1),
    ])
    return (src.replace('@@DEFS@@', defs)
               .replace('@@RHS@@', rhs_body(t))
               .replace('@@COUNTS@@', counts_body(t))
               .replace('@@INVKM@@', invkm_body(t)))
