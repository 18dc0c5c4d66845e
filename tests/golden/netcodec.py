"""JSON codec for convenience-kinetics networks (tuple keys <-> lists).

A species key ``(port, name)`` is stored as ``[port, name]``; parameter names
are either strings (``kcat_f``) or species keys.
"""


def _key_out(k):
    return list(k) if isinstance(k, tuple) else k


def _key_in(k):
    return tuple(k) if isinstance(k, list) else k


def encode_network(reactions, kinetic_parameters):
    rx = {}
    for rid, spec in reactions.items():
        rx[rid] = {
            'stoichiometry': [[_key_out(m), c] for m, c in spec['stoichiometry'].items()],
            'is reversible': bool(spec.get('is reversible', False)),
            'catalyzed by': [_key_out(e) for e in spec['catalyzed by']],
        }
    kp = {}
    for rid, enzymes in kinetic_parameters.items():
        kp[rid] = [[_key_out(e), [[_key_out(p), v] for p, v in params.items()]]
                   for e, params in enzymes.items()]
    return {'reactions': rx, 'kinetic_parameters': kp}


def decode_network(obj):
    reactions = {}
    for rid, spec in obj['reactions'].items():
        reactions[rid] = {
            'stoichiometry': {_key_in(m): c for m, c in spec['stoichiometry']},
            'is reversible': spec['is reversible'],
            'catalyzed by': [_key_in(e) for e in spec['catalyzed by']],
        }
    kinetic_parameters = {}
    for rid, enzymes in obj['kinetic_parameters'].items():
        kinetic_parameters[rid] = {
            _key_in(e): {_key_in(p): v for p, v in params} for e, params in enzymes}
    return reactions, kinetic_parameters


def encode_conc(conc):
    return [[_key_out(k), v] for k, v in conc.items()]


def decode_conc(items):
    return {_key_in(k): v for k, v in items}
