"""The rate-law code generator emits HIP that compiles for gfx950 (no GPU needed)
and evaluates the same rate law as the compiled table."""

import os
import subprocess

import numpy as np
import pytest

from netcodec import decode_network, decode_conc
from lens_amd import configs
from lens_amd.codegen import dopri5_source, rhs_body
from lens_amd.rate_law_compiler import compile_rate_laws


def _hipcc_compile(src, tmp_path):
    f = tmp_path / 'spec.hip'
    f.write_text(src)
    r = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-ffp-contract=off',
                        '-std=c++17', '--cuda-device-only', '-c', str(f), '-o', str(tmp_path / 'spec.o')],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize('name', ['glc_lct', 'glc_ac', 'synthetic'])
def test_generated_source_compiles_for_gfx950(name, tmp_path):
    cfg = {'glc_lct': configs.glc_lct_config, 'glc_ac': configs.glc_ac_config,
           'synthetic': lambda: configs.synthetic_network(n_species=20, n_reactions=12, n_enzymes=4)}[name]()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    _hipcc_compile('#include <hip/hip_runtime.h>\n' + dopri5_source(t), tmp_path)


def _py_rhs(t, conc, params):
    """Evaluate the generated rhs body in Python (same expression text)."""
    p = params.copy()
    for q in set(int(x) for x in t.mem_param):
        p[q] = 1.0 / p[q] if p[q] != 0 else 0.0
    c = list(conc)
    dy = [0.0] * (t.n_dyn + t.n_reactions)
    env = {'c': c, 'p': p, 'dy': dy, 'fma': lambda a, b, d: a * b + d, 'vk_div': lambda a, b: a / b}
    code = []
    for line in rhs_body(t).splitlines():
        s = line.strip()
        if s.startswith('//') or s in ('{', '}') or s.startswith('{  //'):
            continue
        s = s.replace('double ', '').rstrip(';')
        code.append(s)
    exec('\n'.join(code), env)
    return np.array(env['dy'])


def test_generated_rhs_matches_reference_fluxes(golden_fluxes):
    for case in golden_fluxes['cases'][:8]:
        rx, kp = decode_network(case['network'])
        t = compile_rate_laws(rx, kp)
        for conc_items, expect in zip(case['concs'][:4], case['fluxes'][:4]):
            conc = decode_conc(conc_items)
            cv = np.array([float(conc.get(k, 0.0)) for k in t.species])
            dy = _py_rhs(t, cv, t.param_defaults.copy())
            got = dy[t.n_dyn:]
            ref = np.array([expect[r] for r in t.reaction_ids])
            np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize('wpe,pad,lds,split', [(2, 0, 0, 0), (2, 1, 0, 0), (3, 1, 1, 0), (3, 1, 2, 0), (2, 1, 0, 1),
                                              (3, 0, 0, 1)])
def test_wave_source_compiles_for_gfx950(wpe, pad, lds, split, tmp_path):
    """The agent-per-wavefront template (C5 network) in every option
    combination the engine can select: occupancy, branch-free publishes, LDS
    operand tables (levels 1 and 2).  hiprtc compiles the same text at run
    time on the GPU; this catches template errors on the CPU."""
    from lens_amd.codegen import wave_source
    cfg = configs.synthetic_network()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    _hipcc_compile('#include <hip/hip_runtime.h>\n' + wave_source(t, wpe, pad, lds, split), tmp_path)


def test_split_layout():
    """codegen.split_layout on C5: the min(nl, 64 - nl) rate laws with the most
    denominator sets take lanes l and l + 32, each half a contiguous run of
    sets (first half ceil(n/2), summed in lane l); every rate law is written by
    exactly one lane."""
    from lens_amd.codegen import split_layout
    cfg = configs.synthetic_network(n_species=50, n_reactions=40, n_enzymes=10)
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    lanes, dst, second, sets = split_layout(t)
    nl = t.n_rate_laws
    assert sorted(d for d in dst if d >= 0) == list(range(nl))
    nden = [int(t.rl_den_ptr[l + 1] - t.rl_den_ptr[l]) for l in range(nl)]
    P = sum(second)
    assert P == min(nl, 64 - nl)
    for b in range(32, 64):
        if second[b]:
            a = b - 32
            l = lanes[a]
            assert lanes[b] == l and not second[a] and dst[a] == l and dst[b] == -1
            assert sets[a][0] == int(t.rl_den_ptr[l]) and sets[a][1] == sets[b][0]
            assert sets[b][1] == int(t.rl_den_ptr[l + 1]) and sets[a][1] - sets[a][0] == (nden[l] + 1) // 2
    heavy = {lanes[b] for b in range(32, 64) if second[b]}
    assert min(nden[l] for l in heavy) >= max([nden[l] for l in range(nl) if l not in heavy] or [0])
    assert max(hi - lo for lo, hi in sets) == 4     # C5: 6 sets x 3 members -> 4 x 3
