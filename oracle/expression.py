"""Oracle for ODE gene expression -- TEST INFRASTRUCTURE ONLY.

Restates ``ODE_expression.next_update`` (vivarium/processes/ode_expression.py:
265-303) and the boolean regulation language of
vivarium/library/regulation_logic.py (arpeggio grammar :19-27, evaluation
:29-98): ``rule = 'if' logic``; ``logic = term (('and'|'or') logic)?`` evaluated
right-recursively (``a and b or c`` is ``a and (b or c)``); ``term = ['not']
(compare | '[' logic ']')``; ``compare = (symbol | (port, name)) [('>'|'<')
symbol]`` where a lone numeric operand means ``> 0``.  Symbols are looked up in
the tuple-keyed state first and otherwise read as numbers.

The transcription leak draws ``random.uniform(0, 1)`` only for inhibited genes;
``leak(gene)`` supplies that draw here (``None`` = the reference's rate-0
default, where the draw can never pass).
"""

from __future__ import annotations

import math
import re

_TOKEN = re.compile(r'\s*(\(|\)|\[|\]|,|>|<|[a-zA-Z0-9.\-_]+)')
_KEYWORDS = ('if', 'not', 'and', 'or')


def tokenize(text):
    pos, out = 0, []
    text = text.strip()
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise SyntaxError('bad rule near %r' % text[pos:])
        out.append(m.group(1))
        pos = m.end()
    return out


class _Parser:
    def __init__(self, tokens):
        self.t = tokens
        self.i = 0

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else None

    def take(self, want=None):
        tok = self.peek()
        if tok is None or (want is not None and tok != want):
            raise SyntaxError('expected %r, got %r' % (want, tok))
        self.i += 1
        return tok

    def rule(self):
        self.take('if')
        tree = self.logic()
        if self.peek() is not None:
            raise SyntaxError('trailing %r' % self.peek())
        return tree

    def logic(self):
        head = self.term()
        if self.peek() in ('and', 'or'):
            op = self.take()
            return (op, head, self.logic())
        return head

    def term(self):
        if self.peek() == 'not':
            self.take()
            return ('not', self.operand())
        return self.operand()

    def operand(self):
        if self.peek() == '[':
            self.take('[')
            inner = self.logic()
            self.take(']')
            return inner
        if self.peek() == '(':
            self.take('(')
            port = self.take()
            self.take(',')
            name = self.take()
            self.take(')')
            first = ('key', (port, name))
        else:
            first = ('sym', self.take())
        if self.peek() in ('>', '<'):
            op = self.take()
            return ('cmp', first, op, ('sym', self.take()))
        return ('cmp', first, None, None)


def parse(rule):
    return _Parser(tokenize(rule)).rule()


def _value(node, state):
    kind, v = node
    if kind == 'key':
        return state.get(v)
    got = state.get(v)
    if got is None:
        try:
            return float(v)
        except ValueError:
            return None
    return got


def evaluate(tree, state):
    op = tree[0]
    if op == 'not':
        return not evaluate(tree[1], state)
    if op in ('and', 'or'):
        head = evaluate(tree[1], state)
        tail = evaluate(tree[2], state)
        return (head and tail) if op == 'and' else (head or tail)
    _, first, cmp, last = tree
    a = _value(first, state)
    if cmp is None:
        return a > 0 if isinstance(a, (int, float)) else a
    b = _value(last, state)
    return a < b if cmp == '<' else a > b


def next_update(config, timestep, states, leak=None):
    """ODE_expression.next_update on one agent: {'internal': {state: delta}}."""
    internal = states['internal']
    flat = {}
    for port, values in states.items():
        for k, v in values.items():
            flat[(port, k)] = v
    regulation = {g: evaluate(parse(r), flat) for g, r in config.get('regulation', {}).items()}
    leak_cfg = config.get('transcription_leak', {'rate': 0.0, 'magnitude': 0.0})
    degradation = config.get('degradation_rates', {})
    update = {}
    for transcript, rate in config.get('transcription_rates', {}).items():
        m = internal[transcript]
        if transcript in regulation and regulation.get(transcript):
            r = -math.log(1 - leak_cfg['rate'])
            p = 1 - math.exp(-r * timestep)
            u = leak(transcript) if leak is not None else 1.0
            rate = leak_cfg['magnitude'] if u < p else 0.0
        update[transcript] = (rate - degradation.get(transcript, 0) * m) * timestep
    for protein, rate in config.get('translation_rates', {}).items():
        m = internal[config['protein_map'][protein]]
        p_state = internal[protein]
        update[protein] = (rate * m - degradation.get(protein, 0) * p_state) * timestep
    return {'internal': update}
