"""ODE gene expression + boolean regulation.

Pins: the reference's own known answers -- regulation_logic.test_arpeggio
(vivarium/library/regulation_logic.py:118-152) and the ODE_expression doctest
(vivarium/processes/ode_expression.py:124-167) -- for the oracle and the
product's rule compiler; the GPU kernel bit-exact against the oracle."""

import numpy as np
import pytest

from oracle import expression as oe

ARPEGGIO = [
    ('if not [GLCxt or LCTSxt or RUBxt] and FNR and not GlpR',
     {'GLCxt': True, 'LCTSxt': False, 'RUBxt': True, 'FNR': True, 'GlpR': False}, False),
    ('if not [GLCxt or LCTSxt or RUBxt] and FNR and not GlpR',
     {'GLCxt': False, 'LCTSxt': False, 'RUBxt': False, 'FNR': True, 'GlpR': False}, True),
    ('if not glc > 0.1', {'glc': 0.2}, False),
    ('if not glc > 0.1', {'glc': 0.01}, True),
    ('if not [FDP > 10 and F6P]', {'FDP': 20, 'F6P': 10}, False),
    ('if not [FDP > 10 and F6P]', {'FDP': 20, 'F6P': 0}, True),
]


@pytest.mark.parametrize('rule,state,want', ARPEGGIO)
def test_oracle_rules_match_reference_known_answers(rule, state, want):
    assert oe.evaluate(oe.parse(rule), state) == want


def lacy_doctest_config():
    return {
        'transcription_rates': {'lacy_RNA': 3.0}, 'translation_rates': {'LacY': 4.0},
        'degradation_rates': {'lacy_RNA': 1.0, 'LacY': 0.0}, 'protein_map': {'LacY': 'lacy_RNA'},
        'initial_state': {'internal': {'lacy_RNA': 0.0, 'LacY': 0.0}, 'external': {'glc__D_e': 2.0}},
        'regulators': [('external', 'glc__D_e')],
        'regulation': {'lacy_RNA': 'if (external, glc__D_e) > 1.0'},
    }


DOCTEST = [  # (lacy_RNA, glc__D_e) -> reference update (ode_expression.py:157-167)
    ((0.0, 2.0), {'lacy_RNA': 0.0, 'LacY': 0.0}),
    ((1.0, 2.0), {'lacy_RNA': -1.0, 'LacY': 4.0}),
    ((1.0, 0.5), {'lacy_RNA': 2.0, 'LacY': 4.0}),
]


@pytest.mark.parametrize('inp,want', DOCTEST)
def test_oracle_matches_reference_doctest(inp, want):
    states = {'internal': {'lacy_RNA': inp[0], 'LacY': 0.0}, 'external': {'glc__D_e': inp[1]}}
    assert oe.next_update(lacy_doctest_config(), 1, states) == {'internal': want}


def test_compiler_postfix_matches_oracle_on_random_states():
    """The product's compiled programs, interpreted on the host, agree with the
    oracle's tree evaluation (same right-recursive and/or)."""
    from lens_amd.expression import compile_rule, parse_rule, EXPR_CMP_GT, EXPR_CMP_LT, EXPR_PRESENT, \
        EXPR_CONST, EXPR_NOT, EXPR_AND
    keys = [('internal', 'a'), ('internal', 'b'), ('external', 'c')]
    rules = ['if (internal, a) > 0.5 and (external, c) < 2 or not (internal, b)',
             'if not [(internal, a) > 0.1 or (internal, b) < 0.3] and (external, c)',
             'if [(internal, a) > 0.5 and [(internal, b) > 0.5 or not (external, c) > 1.5]]',
             'if 3 > 2 and (internal, b) > 0.2']
    rng = np.random.default_rng(3)
    for rule in rules:
        thr = []
        code = compile_rule(parse_rule(rule), keys.index, thr)
        for _ in range(200):
            vals = rng.uniform(-0.5, 3.0, 3) * (rng.random(3) > 0.2)
            state = {k: float(v) for k, v in zip(keys, vals)}
            stack = []
            for op, x, y in code:
                if op == EXPR_NOT:
                    stack[-1] = not stack[-1]
                elif op in (EXPR_AND, 6):
                    r, l = stack.pop(), stack.pop()
                    stack.append((l and r) if op == EXPR_AND else (l or r))
                elif op == EXPR_CMP_GT:
                    stack.append(vals[x] > thr[y])
                elif op == EXPR_CMP_LT:
                    stack.append(vals[x] < thr[y])
                elif op == EXPR_PRESENT:
                    stack.append(vals[x] > 0)
                elif op == EXPR_CONST:
                    stack.append(bool(x))
            assert bool(stack[-1]) == bool(oe.evaluate(oe.parse(rule), state)), (rule, vals)


torch = pytest.importorskip('torch')


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda', 0)


@pytest.mark.gpu
@pytest.mark.parametrize('inp,want', DOCTEST)
def test_gpu_process_drop_in_reproduces_doctest(dev, inp, want):
    from lens_amd.expression import BatchedODEExpression
    proc = BatchedODEExpression(lacy_doctest_config())
    assert proc.name == 'ode_expression'
    state = {'internal': {'lacy_RNA': 0.0, 'LacY': 0.0}, 'external': {'glc__D_e': 2.0}}
    assert {p: {k: v['_default'] for k, v in d.items()} for p, d in proc.ports_schema().items()
            if p in ('internal', 'external')} == state
    states = {'internal': {'lacy_RNA': inp[0], 'LacY': 0.0}, 'external': {'glc__D_e': inp[1]}}
    assert proc.next_update(1, states) == {'internal': want}


@pytest.mark.gpu
def test_gpu_colony_bitexact_vs_oracle_with_leaks(dev):
    from lens_amd.expression import ExpressionEngine, ExpressionTable
    cfg = {
        'transcription_rates': {'lacy_RNA': 1e-7, 'flag_RNA': 1e-6, 'x_RNA': 2e-6},
        'translation_rates': {'LacY': 5e-3, 'flagella': 8e-5, 'X': 1e-3},
        'degradation_rates': {'lacy_RNA': 3e-3, 'LacY': 3e-5, 'flag_RNA': 2e-2, 'X': 1e-4},
        'protein_map': {'LacY': 'lacy_RNA', 'flagella': 'flag_RNA', 'X': 'x_RNA'},
        'regulators': [('external', 'glc__D_e'), ('internal', 'lcts_p')],
        'regulation': {'lacy_RNA': 'if (external, glc__D_e) > 0.1 and (internal, lcts_p) < 0.01',
                       'x_RNA': 'if not [(internal, LacY) > 1e-6 or (external, glc__D_e) < 4]'},
        'transcription_leak': {'rate': 1e-1, 'magnitude': 1e-6},
    }
    keys = [('internal', k) for k in ('lacy_RNA', 'flag_RNA', 'x_RNA', 'LacY', 'flagella', 'X', 'lcts_p')]
    keys += [('external', 'glc__D_e')]
    t = ExpressionTable(cfg, keys)
    n = 3000
    rng = np.random.default_rng(11)
    conc = rng.uniform(0, 1e-5, (len(keys), n))
    conc[keys.index(('internal', 'lcts_p'))] = rng.choice([0.0, 0.005, 0.05], n)
    conc[keys.index(('external', 'glc__D_e'))] = rng.uniform(0, 8, n)
    u = rng.random((len(t.transcripts), n))
    eng = ExpressionEngine(t, dev)
    c_dev = torch.from_numpy(conc.copy()).to(dev)
    upd = eng.step(1.0, c_dev, u=torch.from_numpy(u).to(dev)).cpu().numpy()
    got_conc = c_dev.cpu().numpy()
    for a in range(n):
        states = {'internal': {}, 'external': {}}
        for r, (port, name) in enumerate(keys):
            states[port][name] = float(conc[r, a])
        draws = dict(zip(t.transcripts, u[:, a]))
        want = oe.next_update(cfg, 1.0, states, leak=lambda g: draws[g])['internal']
        assert [float(x) for x in upd[:, a]] == [want[k] for k in t.outputs], a
    # accumulate updater
    for j, name in enumerate(t.outputs):
        r = keys.index(('internal', name))
        assert np.array_equal(got_conc[r], conc[r] + upd[j])
