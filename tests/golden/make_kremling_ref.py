"""Generate tests/golden/kremling_ref.npz from the REFERENCE's own Kremling code
(TEST FIXTURE GENERATOR; run here, where /root/reference exists -- the GPU box
and the tests only read the committed .npz).

vivarium/processes/Kremling2007_transport.py does not import in this container
for ordinary reasons (its module imports vivarium.core and matplotlib; SURVEY.md
§1.3).  Its model is self-contained, though, so this script reads the file's
AST and evaluates only three pieces of it, unchanged, with numpy and scipy:

* ``DEFAULT_PARAMETERS`` (:19-70), the dict expression evaluated without builtins;
* the state key order, the keys of ``combined_state`` in ``next_update`` (:361-379);
* ``model(state, t)``, the closure inside ``next_update`` (:220-351), compiled
  as a module-level function whose free names ``p`` and ``state_keys`` are the
  two above.

With them it records, for 48 seeded states in each regime of the model's
switch on internal G6P (> 0.01: G6P uptake; else lactose):

* ``dy``: the reference right-hand side at every state;
* ``end_tight`` / ``flux_tight``: odeint (LSODA) of the reference ``model``
  over the reference's own grid ``np.arange(0, 1/3600, 0.01/3600)`` (:354-357,
  :384) at rtol 1e-13 / atol 1e-16 -- the last row (internal species, :409) and
  the mean of the flux integrals (:404), for 12 of the states;
* ``end_default`` / ``flux_default``: the same call at odeint's default
  tolerances, i.e. the reference's literal call.

No reference source is copied into the repository: the file is parsed at
generation time only.  The reference is untrusted input, so nothing of it runs
before an AST whitelist has passed it (``_check_params`` / ``_check_model``):
the parameters may only be a dict of numeric constants and arithmetic on them;
the model only arithmetic, comparisons, subscripts, assignments, ``if`` and
``return``, calls to ``np.zeros_like`` and ``state_keys.index``, and names that
are its own locals, its argument, ``p``, ``state_keys`` or ``np``.  Both are
then evaluated with an empty ``__builtins__``.

    python tests/golden/make_kremling_ref.py
"""

from __future__ import annotations

import ast
import os
import sys

import numpy as np
from scipy.integrate import odeint

REF = '/root/reference/vivarium/processes/Kremling2007_transport.py'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'kremling_ref.npz')


_ARITH = (ast.Add, ast.Sub, ast.Mult, ast.Div, ast.Pow, ast.USub, ast.UAdd)
_CALLS = {('np', 'zeros_like'), ('state_keys', 'index')}


def _check_params(expr):
    """DEFAULT_PARAMETERS: a dict literal of string keys and numeric constants,
    with arithmetic on constants allowed (e.g. 2.4 * 60)."""
    for n in ast.walk(expr):
        ok = isinstance(n, (ast.Dict, ast.Constant, ast.BinOp, ast.UnaryOp, ast.Load) + _ARITH)
        if isinstance(n, ast.Constant) and not isinstance(n.value, (int, float, str)):
            ok = False
        if not ok:
            raise ValueError('DEFAULT_PARAMETERS: disallowed node %s' % ast.dump(n)[:80])


def _check_model(fn):
    """model(state, t): arithmetic over names, subscripts and the two calls in
    _CALLS; every name is an argument, a local it assigns, or p / state_keys / np."""
    args = {a.arg for a in fn.args.args}
    local = {t.id for n in ast.walk(fn) if isinstance(n, ast.Assign) for t in n.targets if isinstance(t, ast.Name)}
    names = args | local | {'p', 'state_keys', 'np'}
    allowed = (ast.FunctionDef, ast.arguments, ast.arg, ast.Assign, ast.Return, ast.If, ast.Expr, ast.Compare,
               ast.BinOp, ast.UnaryOp, ast.Name, ast.Load, ast.Store, ast.Constant, ast.Subscript, ast.Call,
               ast.Attribute, ast.Gt, ast.Lt, ast.GtE, ast.LtE) + _ARITH
    for n in ast.walk(fn):
        if not isinstance(n, allowed):
            raise ValueError('model: disallowed node %s' % type(n).__name__)
        if isinstance(n, ast.Name) and n.id not in names:
            raise ValueError('model: unknown name %s' % n.id)
        if isinstance(n, ast.Attribute):
            if not (isinstance(n.value, ast.Name) and (n.value.id, n.attr) in _CALLS):
                raise ValueError('model: disallowed attribute %s' % ast.unparse(n))
        if isinstance(n, ast.Call):
            if not (isinstance(n.func, ast.Attribute) and isinstance(n.func.value, ast.Name) and
                    (n.func.value.id, n.func.attr) in _CALLS) or n.keywords:
                raise ValueError('model: disallowed call %s' % ast.unparse(n))
        if isinstance(n, ast.Constant) and not isinstance(n.value, (int, float, str)):
            raise ValueError('model: disallowed constant %r' % (n.value,))
        if isinstance(n, ast.Expr) and not isinstance(n.value, ast.Constant):   # docstrings only
            raise ValueError('model: disallowed statement %s' % ast.unparse(n))


def _pieces(path):
    tree = ast.parse(open(path).read(), path)
    params = keys = model = None
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(getattr(t, 'id', None) == 'DEFAULT_PARAMETERS' for t in node.targets):
            _check_params(node.value)
            params = eval(compile(ast.Expression(node.value), path, 'eval'), {'__builtins__': {}})
        if isinstance(node, ast.ClassDef) and node.name == 'Transport':
            nu = next(f for f in node.body if isinstance(f, ast.FunctionDef) and f.name == 'next_update')
            model = next(f for f in nu.body if isinstance(f, ast.FunctionDef) and f.name == 'model')
            for st in nu.body:
                if isinstance(st, ast.Assign) and getattr(st.targets[0], 'id', None) == 'combined_state':
                    keys = [k.value for k in st.value.keys]
    assert params and keys and model, 'reference layout changed'
    _check_model(model)
    mod = ast.Module(body=[model], type_ignores=[])
    ns = {'__builtins__': {}, 'np': np, 'p': dict(params), 'state_keys': list(keys)}
    exec(compile(mod, path, 'exec'), ns)
    return ns['model'], params, keys


def main():
    model, params, keys = _pieces(REF)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from oracle import kremling as ok
    assert tuple(keys) == ok.STATE_KEYS, keys
    rng = np.random.default_rng(2026_10_17)
    states = []
    for regime, (internal, external) in enumerate(((ok.GLC_G6P_INTERNAL, ok.GLC_G6P_EXTERNAL),
                                                   (ok.GLC_LCT_SHIFT_INTERNAL, ok.GLC_LCT_SHIFT_EXTERNAL))):
        s0 = ok.initial_state(internal, external)
        for i in range(48):
            s = s0.copy()
            if i:
                s[:8] *= rng.uniform(0.6, 1.4, 8)
                s[8:11] *= rng.uniform(0.5, 1.5, 3)
                s[11:] = rng.uniform(0.0, 1e-3, 4) if i % 2 else 0.0
            if regime:       # the lactose branch: internal G6P at or below the 0.01 switch (:245)
                s[4] = 0.01 * (rng.uniform(0.1, 1.0) if i else 0.5)
                s[2] = max(s[2], 1e-5 * rng.uniform(0.5, 2.0))   # some LACZ to take up lactose
            states.append(s)
    states = np.array(states)                                     # [96, 15]
    dy = np.array([model(s, 0.0) for s in states])
    t = np.arange(0, 1.0 / 3600, 0.01 / 3600)
    pick = np.r_[0:6, 48:54]                                      # 6 states per regime
    end_tight, flux_tight, end_default, flux_default = [], [], [], []
    for i in pick:
        s = states[i].copy()
        s[11:] = 0.0                                             # next_update starts the integrals at 0 (:375-378)
        sol = odeint(model, s, t, rtol=1e-13, atol=1e-16, mxstep=500000)
        end_tight.append(sol[-1, :8])
        flux_tight.append([np.mean(sol[:, c]) for c in range(11, 15)])     # per column, as :404
        lit = odeint(model, s, t)
        end_default.append(lit[-1, :8])
        flux_default.append([np.mean(lit[:, c]) for c in range(11, 15)])
    np.savez_compressed(OUT, states=states, dy=dy, pick=pick, end_tight=np.array(end_tight),
                        flux_tight=np.array(flux_tight), end_default=np.array(end_default),
                        flux_default=np.array(flux_default),
                        keys=np.array(keys), params=np.array([params[k] for k in sorted(params)], dtype=np.float64),
                        param_names=np.array(sorted(params)))
    print('wrote', OUT, states.shape, 'regimes', int((states[:, 4] > 0.01).sum()), int((states[:, 4] <= 0.01).sum()))


if __name__ == '__main__':
    main()
