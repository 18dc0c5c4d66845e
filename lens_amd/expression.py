"""Batched ODE gene expression with boolean regulation.

``ODE_expression`` (vivarium/processes/ode_expression.py:29-303) advances, per
agent and timestep, transcripts ``dM = (k_M - d_M*M)*dt`` (zero -- or the leak
magnitude -- while the transcript's regulation rule holds) and proteins
``dP = (k_P*m - d_P*P)*dt``.  Rules are strings in the language of
vivarium/library/regulation_logic.py (``'if (external, glc__D_e) > 0.1 and
not [(internal, lcts_p) < 0.01]'``).

Here a rule is parsed once (same grammar, same right-recursive and/or
evaluation) and compiled to a postfix program over the agent's state rows;
``vk_expression_step`` evaluates every agent's rules and updates in one launch.
:class:`BatchedODEExpression` is the Process-API drop-in (same ``name``,
``defaults``, ``ports_schema``, ``next_update``).
"""

from __future__ import annotations

import ctypes
import math
import re
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from lens_amd import native
from lens_amd.process import ProcessBase, deep_merge

EXPR_CMP_GT, EXPR_CMP_LT, EXPR_PRESENT, EXPR_CONST, EXPR_NOT, EXPR_AND, EXPR_OR = range(7)

_TOKEN = re.compile(r'\s*(\(|\)|\[|\]|,|>|<|[a-zA-Z0-9.\-_]+)')


class RuleSyntaxError(SyntaxError):
    pass


def _tokens(text):
    pos, out, text = 0, [], text.strip()
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise RuleSyntaxError('bad rule near %r' % text[pos:])
        out.append(m.group(1))
        pos = m.end()
    return out


def parse_rule(text):
    """regulation_logic.py grammar (:19-27) -> nested tuples:
    ('and'|'or', lhs, rhs) | ('not', x) | ('cmp', first, op|None, threshold|None)
    with first = ('key', (port, name)) | ('num', value)."""
    toks = _tokens(text)
    i = [0]

    def peek():
        return toks[i[0]] if i[0] < len(toks) else None

    def take(want=None):
        t = peek()
        if t is None or (want is not None and t != want):
            raise RuleSyntaxError('expected %r, got %r in %r' % (want, t, text))
        i[0] += 1
        return t

    def logic():
        head = term()
        if peek() in ('and', 'or'):
            op = take()
            return (op, head, logic())          # right-recursive, as evaluate_logic
        return head

    def term():
        if peek() == 'not':
            take()
            return ('not', operand())
        return operand()

    def number(tok):
        try:
            return float(tok)
        except ValueError:
            raise RuleSyntaxError('%r is neither a (port, name) key nor a number in %r' % (tok, text))

    def operand():
        if peek() == '[':
            take('[')
            inner = logic()
            take(']')
            return inner
        if peek() == '(':
            take('(')
            port = take()
            take(',')
            name = take()
            take(')')
            first = ('key', (port, name))
        else:
            first = ('num', number(take()))
        if peek() in ('>', '<'):
            op = take()
            return ('cmp', first, op, number(take()))
        return ('cmp', first, None, None)

    take('if')
    tree = logic()
    if peek() is not None:
        raise RuleSyntaxError('trailing %r in %r' % (peek(), text))
    return tree


def compile_rule(tree, row_of, thresholds: List[float]) -> List[Tuple[int, int, int]]:
    """Postfix [op, a, b] triples; row_of maps (port, name) -> state row."""
    out: List[Tuple[int, int, int]] = []

    def emit(node):
        kind = node[0]
        if kind == 'not':
            emit(node[1])
            out.append((EXPR_NOT, 0, 0))
        elif kind in ('and', 'or'):
            emit(node[1])
            emit(node[2])
            out.append((EXPR_AND if kind == 'and' else EXPR_OR, 0, 0))
        else:
            _, first, op, thr = node
            if first[0] == 'num':
                a = first[1]
                value = (a > thr if op == '>' else a < thr) if op else a > 0
                out.append((EXPR_CONST, int(bool(value)), 0))
                return
            row = row_of(first[1])
            if op is None:
                out.append((EXPR_PRESENT, row, 0))
            else:
                thresholds.append(float(thr))
                out.append((EXPR_CMP_GT if op == '>' else EXPR_CMP_LT, row, len(thresholds) - 1))

    emit(tree)
    return out


class ExpressionTable:
    """A compiled ODE_expression configuration over state rows ``keys``."""

    def __init__(self, config, keys: Sequence[Tuple[str, str]]):
        self.keys = [tuple(k) for k in keys]
        index = {k: r for r, k in enumerate(self.keys)}

        def row_of(key):
            if tuple(key) not in index:
                raise KeyError('regulation refers to %r, which is not a state row' % (key,))
            return index[tuple(key)]

        deg = config.get('degradation_rates', {})
        self.transcripts = list(config.get('transcription_rates', {}).keys())
        self.proteins = list(config.get('translation_rates', {}).keys())
        reg = config.get('regulation', {})
        thresholds: List[float] = []
        prog_ptr, code = [0], []
        for tname in self.transcripts:
            if tname in reg:
                code += compile_rule(parse_rule(reg[tname]), row_of, thresholds)
            prog_ptr.append(len(code))
        self.tx_row = np.array([row_of(('internal', t)) for t in self.transcripts], dtype=np.int32)
        self.tx_rate = np.array([config['transcription_rates'][t] for t in self.transcripts], dtype=np.float64)
        self.tx_deg = np.array([deg.get(t, 0) for t in self.transcripts], dtype=np.float64)
        self.tx_prog_ptr = np.array(prog_ptr, dtype=np.int32)
        self.code = np.array(code, dtype=np.int32).reshape(-1) if code else np.zeros(3, dtype=np.int32)
        self.thr = np.array(thresholds or [0.0], dtype=np.float64)
        pmap = config.get('protein_map', {})
        self.tl_row = np.array([row_of(('internal', p)) for p in self.proteins], dtype=np.int32)
        self.tl_mrna_row = np.array([row_of(('internal', pmap[p])) for p in self.proteins], dtype=np.int32)
        self.tl_rate = np.array([config['translation_rates'][p] for p in self.proteins], dtype=np.float64)
        self.tl_deg = np.array([deg.get(p, 0) for p in self.proteins], dtype=np.float64)
        leak = config.get('transcription_leak', {'rate': 0.0, 'magnitude': 0.0})
        self.leak_rate = float(leak['rate'])
        self.leak_magnitude = float(leak['magnitude'])

    def leak_probability(self, dt: float) -> float:
        """ode_expression.py:281-282, evaluated as the reference does."""
        rate = -math.log(1 - self.leak_rate)
        return 1 - math.exp(-rate * dt)

    @property
    def outputs(self):
        return self.transcripts + self.proteins


class VkExprTable(ctypes.Structure):
    _p = ctypes.c_void_p
    _fields_ = [('n_tx', ctypes.c_int32), ('n_tl', ctypes.c_int32),
                ('tx_row', _p), ('tx_rate', _p), ('tx_deg', _p), ('tx_prog_ptr', _p), ('code', _p), ('thr', _p),
                ('tl_row', _p), ('tl_mrna_row', _p), ('tl_rate', _p), ('tl_deg', _p),
                ('leak_p', ctypes.c_double), ('leak_magnitude', ctypes.c_double)]


class ExpressionEngine:
    """An ExpressionTable resident on one GPU."""

    def __init__(self, table: ExpressionTable, device=None):
        native.load()
        self.table = table
        self.device = native.resolve_device(device)
        self._dev = {k: torch.from_numpy(np.ascontiguousarray(getattr(table, k))).to(self.device)
                     for k in ('tx_row', 'tx_rate', 'tx_deg', 'tx_prog_ptr', 'code', 'thr', 'tl_row',
                               'tl_mrna_row', 'tl_rate', 'tl_deg')}

    def step(self, dt, conc, n_agents=None, update=None, u=None, accumulate=True):
        """conc [len(keys), ld] float64 (device).  Returns update [n_tx+n_tl, ld]."""
        t = self.table
        ld = conc.shape[1]
        n = ld if n_agents is None else int(n_agents)
        if conc.dtype != torch.float64 or conc.shape[0] != len(t.keys) or not conc.is_contiguous():
            raise ValueError('conc must be contiguous float64 [%d, ld]' % len(t.keys))
        if update is None:
            update = torch.zeros((len(t.outputs), ld), dtype=torch.float64, device=self.device)
        d = VkExprTable()
        d.n_tx, d.n_tl = len(t.transcripts), len(t.proteins)
        for k, v in self._dev.items():
            setattr(d, k, v.data_ptr())
        d.leak_p = t.leak_probability(dt) if t.leak_rate > 0 else 0.0
        d.leak_magnitude = t.leak_magnitude
        native.check(native._lib.vk_expression_step(
            ctypes.byref(d), n, ld, float(dt), native.ptr(conc), native.ptr(update), native.ptr(u),
            int(bool(accumulate)), native.stream_handle()), 'vk_expression_step')
        return update


class BatchedODEExpression(ProcessBase):
    """Process-API drop-in for ``ODE_expression`` (ode_expression.py:144-303)."""

    name = 'ode_expression'
    defaults = {
        'time_step': 1.0, 'transcription_rates': {}, 'translation_rates': {}, 'degradation_rates': {},
        'protein_map': {}, 'transcription_leak': {'rate': 0.0, 'magnitude': 0.0}, 'regulation': {},
        'regulators': [], 'initial_state': {}, 'counts_deriver_key': 'expression_counts',
    }

    def __init__(self, parameters=None):
        super().__init__(parameters)
        p = self.parameters
        regulators = p.get('regulators')
        self.internal_regulators = [s for port, s in regulators if port == 'internal']
        self.external_regulators = [s for port, s in regulators if port == 'external']
        states = list(p['transcription_rates'].keys()) + list(p['translation_rates'].keys())
        self.initial_state = deep_merge({'internal': {s: 0 for s in states}}, p.get('initial_state'))
        self.internal = list(self.initial_state.get('internal', {}).keys())
        self.external = list(self.initial_state.get('external', {}).keys())
        keys = [('internal', s) for s in dict.fromkeys(self.internal + self.internal_regulators)]
        keys += [('external', s) for s in dict.fromkeys(self.external + self.external_regulators)]
        self.table = ExpressionTable(p, keys)
        self._engine = None

    def ports_schema(self):
        schema = {port: {} for port in ('internal', 'external', 'counts', 'global')}
        for state in self.internal + self.internal_regulators:
            schema['internal'][state] = {'_default': self.initial_state['internal'].get(state, 0.0), '_emit': True}
        for state in self.external + self.external_regulators:
            schema['external'][state] = {'_default': self.initial_state['external'].get(state, 0.0), '_emit': True}
        for state in self.internal + self.internal_regulators:
            schema['counts'][state] = {'_divider': 'split', '_emit': True}
        return schema

    def derivers(self):
        return {self.parameters['counts_deriver_key']: {
            'deriver': 'counts_deriver',
            'port_mapping': {'global': 'global', 'concentrations': 'internal', 'counts': 'counts'},
            'config': {'concentration_keys': self.internal + self.internal_regulators}}}

    def next_update(self, timestep, states, leak_uniforms=None):
        """A batch of one.  ``leak_uniforms`` ({transcript: u}) supplies the
        leak draws the reference takes from ``random.uniform`` (default: no leak)."""
        if self._engine is None:
            self._engine = ExpressionEngine(self.table)
        t = self.table
        col = np.array([[float(getattr(states.get(port, {}).get(name, 0.0), 'magnitude',
                                       states.get(port, {}).get(name, 0.0)))] for port, name in t.keys])
        conc = torch.from_numpy(np.ascontiguousarray(col)).to(self._engine.device)
        u = None
        if leak_uniforms is not None:
            u = torch.tensor([[float(leak_uniforms.get(g, 1.0))] for g in t.transcripts], dtype=torch.float64,
                             device=self._engine.device)
        upd = self._engine.step(timestep, conc, u=u, accumulate=False).cpu().numpy()[:, 0]
        return {'internal': {name: float(v) for name, v in zip(t.outputs, upd)}}
