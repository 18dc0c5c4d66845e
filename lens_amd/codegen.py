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


# ---------------------------------------------------------------------------
# agent-per-wavefront specialisation (vk_dopri5_wave_spec.hip.in)
# ---------------------------------------------------------------------------

WAVE_TEMPLATE = os.environ.get('VK_DOPRI5_WAVE_TEMPLATE') or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), 'csrc', 'vk_dopri5_wave_spec.hip.in')
WAVE_LANES = 64


def wave_shape(t: RateLawTable) -> dict:
    """The padded per-round rate-law shape and the per-lane table sizes."""
    nl, nr, nd = t.n_rate_laws, t.n_reactions, t.n_dyn
    ny = nd + nr

    def sizes(ptr_lo, ptr_hi):
        return [[int(t.set_ptr[s + 1] - t.set_ptr[s]) for s in range(ptr_lo[l], ptr_hi[l])] for l in range(nl)]

    num = sizes(t.rl_num_ptr[:-1], t.rl_num_ptr[1:])
    den = sizes(t.rl_den_ptr[:-1], t.rl_den_ptr[1:])
    per_rx = [[l for l in range(nl) if int(t.rl_reaction[l]) == r] for r in range(nr)]
    upd = [int(t.upd_ptr[i + 1] - t.upd_ptr[i]) for i in range(nd)]
    return {
        'LR': max(1, -(-nl // WAVE_LANES)),
        'SN': max((len(x) for x in num), default=0),
        'MN': max((m for x in num for m in x), default=0),
        'SD': max((len(x) for x in den), default=0),
        'MD': max((m for x in den for m in x), default=0),
        'NSLOT': max(1, -(-ny // WAVE_LANES)),
        'UM': max(upd, default=0),
        'RX_IDENTITY': int(nl == nr and all(int(t.rl_reaction[l]) == l for l in range(nl))),
        'RXR': max(1, -(-nr // WAVE_LANES)),
        'RXM': max((len(x) for x in per_rx), default=0),
        'num': num, 'den': den, 'per_rx': per_rx,
    }


def wave_registers(t: RateLawTable, split: bool = False) -> int:
    """Rough VGPR estimate of the specialised wave kernel (lane constants + DP45 state);
    ``split``: with the split-denominator layout (:func:`split_layout`).  It runs ~30
    under the compiler's count (C5: 180 / 220 one lane per rate law, 162 / 190 split)."""
    s = wave_shape(t)
    lay = split_layout(t) if split else None
    if lay is not None:
        s['SD'] = max(hi - lo for lo, hi in lay[3])
    lane = s['LR'] * (3 * s['SN'] * s['MN'] + 2 * s['SN'] + 1 + 3 * s['SD'] * s['MD']) + s['NSLOT'] * (1 + 3 * s['UM'])
    return lane + 18 * s['NSLOT'] + 40


def _table(name: str, ctype: str, rows) -> str:
    """rows: list over outer dims of lists of 64-lane lists -> a C initializer."""
    def fmt(v):
        return repr(float(v)) if ctype == 'double' else str(int(v))

    def rec(x):
        if isinstance(x, (list, tuple)):
            return '{' + ', '.join(rec(e) for e in x) + '}'
        return fmt(x)

    dims = []
    x = rows
    while isinstance(x, (list, tuple)):
        dims.append(len(x))
        x = x[0] if x else 0
    dims = [max(d, 1) for d in dims]
    if not rows or any(d == 0 for d in dims):
        return '__device__ const %s %s%s = {};' % (ctype, name, ''.join('[%d]' % d for d in dims))
    return '__device__ const %s %s%s = %s;' % (ctype, name, ''.join('[%d]' % d for d in dims), rec(rows))


def split_layout(t: RateLawTable):
    """Lane layout of the split-denominator option (one round of <= 64 rate laws).

    The P = min(nl, 64 - nl, 32) rate laws with the most denominator sets get
    two lanes, l and l + 32: lane l takes the first ceil(n/2) sets and lane
    l + 32 the rest.  Lane l + 32 hands its set terms (term - 1) to lane l over
    v_permlane32_swap, and lane l adds them after its own in set order -- the
    same sequential sum as one lane (kinetic_rate_laws.py:160-172), so the
    result is bit-identical.  The other rate laws keep one lane each, in lanes
    [P, 32) and [32 + P, 64).  Returns (lanes, dst, second, sets): per lane its
    rate law (-1 idle), the rate law it writes (-1: the scratch slot), the
    second-half flag and its (set_lo, set_hi) range; None if not applicable.
    """
    nl, W, H = t.n_rate_laws, WAVE_LANES, WAVE_LANES // 2
    if nl == 0 or nl > W:
        return None
    nden = [int(t.rl_den_ptr[l + 1] - t.rl_den_ptr[l]) for l in range(nl)]
    P = min(nl, W - nl, H)
    if P == 0:
        return None            # 64 rate laws: no lane to spare
    order = sorted(range(nl), key=lambda l: (-nden[l], l))
    heavy = sorted(order[:P])
    single = sorted(order[P:])
    lanes, dst, second = [-1] * W, [-1] * W, [0] * W
    sets = [(0, 0)] * W
    for i, l in enumerate(heavy):
        a, b = i, i + H
        lo, hi = int(t.rl_den_ptr[l]), int(t.rl_den_ptr[l + 1])
        mid = lo + (hi - lo + 1) // 2
        lanes[a] = lanes[b] = l
        dst[a] = l
        second[b] = 1
        sets[a], sets[b] = (lo, mid), (mid, hi)
    free = list(range(P, H)) + list(range(H + P, W))
    for x, l in zip(free, single):
        lanes[x] = dst[x] = l
        sets[x] = (int(t.rl_den_ptr[l]), int(t.rl_den_ptr[l + 1]))
    return lanes, dst, second, sets


def wave_source(t: RateLawTable, wpe: int = 3, pad_writes: int = 0, lds_ops: int = 0, split_den: int = 0,
                group: int = 2) -> str:
    """Complete HIP source of the specialised agent-per-wavefront kernel ``vk_dopri5_wspec``.

    split_den = 1 lays the rate laws out two lanes per heavy denominator
    (:func:`split_layout`): the padded denominator shape shrinks (C5: 6 sets x 3
    members -> 4 x 3) and the kernel fits three waves per SIMD; the sum is the
    table walk's, so results stay bit-identical.  group = agents (waves) per
    workgroup; the launcher reads it back from the kernel's launch bound."""
    sh = wave_shape(t)
    W = WAVE_LANES
    ns, nr, nl, nd = t.n_species, t.n_reactions, t.n_rate_laws, t.n_dyn
    if lds_ops >= 2 and ns + 1 > 32767:
        raise ValueError('lds_ops=2 keeps species indices in 16 bits')
    ny = nd + nr
    lay = split_layout(t) if split_den else None
    if split_den and lay is None:
        raise ValueError('split_den needs one round of <= 64 rate laws')
    SB = 0
    if lay is not None:
        lanes, dst, second, sets = lay
        sh['SD'] = max(hi - lo for lo, hi in sets)
        SB = max([hi - lo for (lo, hi), b in zip(sets, second) if b] or [0])
    LR, SN, MN, SD, MD = sh['LR'], sh['SN'], sh['MN'], sh['SD'], sh['MD']
    PAD_SP = ns   # cl[NS] == 1.0
    spn = [[[PAD_SP] * W for _ in range(max(SN * MN, 1))] for _ in range(LR)]
    pin = [[[-1] * W for _ in range(max(SN * MN, 1))] for _ in range(LR)]
    kc = [[[-1] * W for _ in range(max(SN, 1))] for _ in range(LR)]
    enz = [[PAD_SP] * W for _ in range(LR)]
    spd = [[[PAD_SP] * W for _ in range(max(SD * MD, 1))] for _ in range(LR)]
    pid = [[[-1] * W for _ in range(max(SD * MD, 1))] for _ in range(LR)]
    if lay is None:
        placement = [(l, divmod(l, W), (int(t.rl_den_ptr[l]), int(t.rl_den_ptr[l + 1]))) for l in range(nl)]
    else:
        placement = [(l, (0, x), sets[x]) for x, l in enumerate(lanes) if l >= 0]
    for l, (r, lane), (dlo, dhi) in placement:
        enz[r][lane] = int(t.rl_enzyme[l])
        for si, s in enumerate(range(t.rl_num_ptr[l], t.rl_num_ptr[l + 1])):
            kc[r][si][lane] = int(t.rl_kcat[l])
            for mi, m in enumerate(range(t.set_ptr[s], t.set_ptr[s + 1])):
                spn[r][si * MN + mi][lane] = int(t.mem_species[m])
                pin[r][si * MN + mi][lane] = int(t.mem_param[m])
        for si, s in enumerate(range(dlo, dhi)):
            for mi, m in enumerate(range(t.set_ptr[s], t.set_ptr[s + 1])):
                spd[r][si * MD + mi][lane] = int(t.mem_species[m])
                pid[r][si * MD + mi][lane] = int(t.mem_param[m])
    NSLOT, UM = sh['NSLOT'], sh['UM']
    ui = [[nr] * W for _ in range(NSLOT)]
    ur = [[[nr] * W for _ in range(max(UM, 1))] for _ in range(NSLOT)]
    uc = [[[0.0] * W for _ in range(max(UM, 1))] for _ in range(NSLOT)]
    for i in range(ny):
        k, lane = divmod(i, W)
        if i < nd:
            for j, q in enumerate(range(t.upd_ptr[i], t.upd_ptr[i + 1])):
                ur[k][j][lane] = int(t.upd_rxn[q])
                uc[k][j][lane] = float(t.upd_coeff[q])
        else:
            ui[k][lane] = i - nd
    RXR, RXM = sh['RXR'], sh['RXM']
    rx = [[[nl] * W for _ in range(max(RXM, 1))] for _ in range(RXR)]
    for r, ls in enumerate(sh['per_rx']):
        rr, lane = divmod(r, W)
        for j, l in enumerate(ls):
            rx[rr][j][lane] = l
    tables = '\n'.join([
        _table('T_SPN', 'int', spn), _table('T_PIN', 'int', pin), _table('T_KC', 'int', kc),
        _table('T_ENZ', 'int', enz), _table('T_SPD', 'int', spd), _table('T_PID', 'int', pid),
        _table('T_UI', 'int', ui), _table('T_UR', 'int', ur), _table('T_UC', 'double', uc),
        _table('T_RX', 'int', rx),
    ])
    if lay is not None:
        first = [1 if b < 32 and second[b + 32] else 0 for b in range(W)]
        tables += '\n' + '\n'.join([_table('T_DST', 'int', [dst]), _table('T_FIRST', 'int', [first])])
    defs = '\n'.join('#define %s %d' % (k, v) for k, v in [
        ('NS', ns), ('ND', nd), ('NR', nr), ('NL', nl), ('NY', ny), ('LR', LR), ('SN', SN), ('MN', MN),
        ('SD', SD), ('MD', MD), ('NSLOT', NSLOT), ('UM', UM), ('RX_IDENTITY', sh['RX_IDENTITY']),
        ('RXR', RXR), ('RXM', RXM), ('TILE', ns + 1 + nr + 1 + nl + 1 + (W if pad_writes else 0)), ('WPE', wpe),
        ('PAD_WRITES', int(pad_writes)), ('LDS_OPS', int(lds_ops)), ('SPLIT_DEN', int(lay is not None)), ('SB', SB),
        ('DW_WAVES', int(group))])
    umk = [max([int(t.upd_ptr[i + 1] - t.upd_ptr[i]) for i in range(k * W, min(nd, (k + 1) * W))] or [0])
           for k in range(NSLOT)]
    defs += '\n__device__ constexpr int UMK[NSLOT] = {%s};' % ', '.join(str(u) for u in umk)
    counts = []
    for e in range(t.n_ext):
        terms = ['        c += trunc_count((%s * fl[%d]) * mc, cst);' % (_f(t.ex_coeff[j]), int(t.ex_rxn[j]))
                 for j in range(t.ex_ptr[e], t.ex_ptr[e + 1])]
        counts.append('    if (lane == %d) {\n        i64 c = 0;\n%s\n        counts[(i64)%d * ld + a] = c;\n    }'
                      % (e % W, '\n'.join(terms), e))
    with open(WAVE_TEMPLATE) as f:
        src = f.read()
    return src.replace('@@DEFS@@', defs).replace('@@TABLES@@', tables).replace('@@COUNTS@@', '\n'.join(counts))
