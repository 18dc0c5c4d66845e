"""Division for the Process-API loop (:class:`lens_amd.engine.Experiment`).

Restates what a dividing compartment needs from the reference:

* the divider registry (vivarium/core/registry.py:197-280): ``set``,
  ``split`` (ints: the odd count goes to a random daughter via
  ``random.choice``; ``inf``/``'Infinity'`` kept; floats halved), ``zero``,
  ``split_dict``, ``no_divide``; a schema ``_divider`` may also be a callable
  or ``{'divider': fn, 'topology': {...}}`` (the divider gets the states at
  those paths, relative to the store holding the leaf);
* ``MetaDivision`` (vivarium/processes/meta_division.py:24-88), the deriver
  that turns ``global.divide`` into a ``_divide`` update with the daughters'
  generated processes and topology, ids from ``daughter_phylogeny_id``;
* ``GrowthProtein`` (vivarium/processes/growth_protein.py:20-107), the
  ``growth_division_minimal`` growth process (units removed: masses in fg,
  protein as a count), and the two derivers it asks for (``derivers()``):
  ``TreeMass`` (tree_mass.py:10-65) and ``DeriveGlobals``
  (derive_globals.py:17-150), with the scalars pint produces in the reference
  evaluated as :class:`lens_amd.cells.CellModel` does for the device colony;
* :func:`growth_division_minimal`, the compartment
  (vivarium/compartments/growth_division_minimal.py:22-60 plus
  process.py:75-103's generated derivers, which come first).

The store side (``_divide`` / ``_generate`` / ``_delete`` / ``_add`` in
``Store.apply_update``, experiment.py:628-697) lives in
:meth:`lens_amd.engine.Experiment._structural`.  The device-resident colony
(:class:`lens_amd.colony.Colony`) divides on the GPU instead (vk_divide_*).
"""

from __future__ import annotations

import random

import numpy as np

from lens_amd.process import ProcessBase

# derive_globals.py:16 takes scipy.constants.N_A; the reference fixtures were made
# with scipy < 1.4, i.e. the CODATA-2014 value (SURVEY.md §0 finding 2)
AVOGADRO = 6.022140857e23


def divide_set(state):
    return [state, state]


def divide_split(state):
    """registry.py:205-236 (a bool is an int there too)."""
    if isinstance(state, (int, np.integer)):
        remainder = state % 2
        half = int(state / 2)
        if random.choice([True, False]):
            return [half + remainder, half]
        return [half, half + remainder]
    if state == float('inf') or state == 'Infinity':
        return [state, state]
    if isinstance(state, (float, np.floating)):
        half = state / 2
        return [half, half]
    raise Exception('can not divide state {} of type {}'.format(state, type(state)))


def divide_zero(state):
    return [0, 0]


def divide_split_dict(state):
    """registry.py:246-272: the first half of the keys to one daughter, the rest to the other."""
    if state is None:
        state = {}
    d1 = dict(list(state.items())[len(state) // 2:])
    d2 = dict(list(state.items())[:len(state) // 2])
    return [d1, d2]


def assert_no_divide(state):
    raise AssertionError('division cannot occur during this process')


DIVIDERS = {'set': divide_set, 'split': divide_split, 'split_dict': divide_split_dict, 'zero': divide_zero,
            'no_divide': assert_no_divide}


def daughter_phylogeny_id(mother_id):
    """meta_division.py:15-18."""
    return [str(mother_id) + '0', str(mother_id) + '1']


def divider_set_false(state):
    return [False, False]


class MetaDivision(ProcessBase):
    """meta_division.py:24-88: a deriver; when ``global.divide`` is set it
    returns ``{'cells': {'_divide': {'mother': agent_id, 'daughters': [...]}}}``
    with each daughter's processes and topology from ``compartment`` (an object
    with ``generate(config) -> {'processes', 'topology'}``, or a callable of
    the config)."""

    name = 'meta_division'
    defaults = {'initial_state': {}, 'daughter_path': ('cell',), 'daughter_ids_function': daughter_phylogeny_id}

    def __init__(self, initial_parameters=None):
        initial_parameters = dict(initial_parameters or {})
        self.division = 0
        self.agent_id = initial_parameters['agent_id']
        self.compartment = initial_parameters['compartment']
        self.daughter_ids_function = initial_parameters.get('daughter_ids_function',
                                                            self.defaults['daughter_ids_function'])
        self.daughter_path = tuple(initial_parameters.get('daughter_path', self.defaults['daughter_path']))
        params = {k: v for k, v in initial_parameters.items() if k not in ('compartment', 'daughter_ids_function')}
        super().__init__(params)

    def is_deriver(self):
        return True

    def ports_schema(self):
        return {'global': {'divide': {'_default': False, '_updater': 'set', '_divider': divider_set_false}},
                'cells': {'*': {}}}

    def _generate(self, config):
        gen = getattr(self.compartment, 'generate', None)
        return gen(config) if gen is not None else self.compartment(config)

    def next_update(self, timestep, states):
        if not states['global']['divide']:
            return {}
        daughters = []
        for daughter_id in self.daughter_ids_function(self.agent_id):
            compartment = self._generate({'agent_id': daughter_id})
            daughters.append({'daughter': daughter_id, 'path': (daughter_id,) + self.daughter_path,
                              'processes': compartment['processes'], 'topology': compartment['topology'],
                              'initial_state': {}})
        return {'cells': {'_divide': {'mother': self.agent_id, 'daughters': daughters}}}


class GrowthProtein(ProcessBase):
    """growth_protein.py:20-107 with units removed: the protein count grows by
    exp(rate * dt), the fractional remainder drawn with np.random.random(); the
    cell divides once the count reaches twice the initial protein."""

    name = 'growth_protein'
    defaults = {'initial_mass': 1339.0, 'protein_mw': 2.09e4, 'growth_rate': 0.000275,
                'global_deriver_key': 'global_deriver', 'mass_deriver_key': 'mass_deriver'}

    def __init__(self, initial_parameters=None):
        super().__init__(initial_parameters)
        p = self.parameters
        self.growth_rate = p['growth_rate']
        # (initial_mass fg).to('g') / (protein_mw g/mol) * N_A
        self.initial_protein = p['initial_mass'] * 1e-15 / p['protein_mw'] * AVOGADRO
        self.divide_protein = self.initial_protein * 2

    def ports_schema(self):
        return {'internal': {'protein': {'_default': self.initial_protein, '_divider': 'split', '_emit': True}},
                'global': {'volume': {'_updater': 'set', '_divider': 'split'},
                           'divide': {'_default': False, '_updater': 'set'}}}

    def next_update(self, timestep, states):
        protein = states['internal']['protein']
        total_protein = protein * np.exp(self.parameters['growth_rate'] * timestep)
        new_protein = int(total_protein - protein)
        extra = total_protein - int(total_protein)
        if np.random.random() < extra:
            new_protein += 1
        return {'internal': {'protein': new_protein}, 'global': {'divide': bool(protein >= self.divide_protein)}}



class TreeMass(ProcessBase):
    """tree_mass.py:21-65: the agent's mass = initial_mass + the mass of every
    count whose schema carries a molecular weight (``_properties.mw``), summed
    over the agent's tree in store order (the ``_reduce`` update with
    calculate_mass).  Here the counts with a weight are named by ``mw_paths``
    ({path below the agent: g/mol}); the fg sum is CellModel.tree_mass's."""

    name = 'mass_deriver'
    defaults = {'initial_mass': 0.0, 'mw_paths': {}}

    def __init__(self, initial_parameters=None):
        super().__init__(initial_parameters)
        self.mw_paths = dict(self.parameters['mw_paths'])

    def is_deriver(self):
        return True

    def ports_schema(self):
        init = self.parameters['initial_mass']
        return {'global': {'initial_mass': {'_default': init, '_updater': 'set', '_divider': 'split'},
                           'mass': {'_default': init, '_emit': True, '_updater': 'set', '_divider': 'split'}},
                'agent': {}}

    def next_update(self, timestep, states):
        from lens_amd.cells import FG_PER_G
        value = states['global']['initial_mass']
        agent = states['agent']
        for path, mw in self.mw_paths.items():
            node = agent
            for k in path:
                node = node.get(k) if isinstance(node, dict) else None
            if node is not None:
                # calculate_mass: value + mw * (count / N_A), the g converted to fg
                value = value + (mw * (node / AVOGADRO)) * FG_PER_G
        return {'global': {'mass': value}}


class DeriveGlobals(ProcessBase):
    """derive_globals.py:54-150: volume, mmol_to_counts, length, surface area and
    periplasm volume from the mass (capsule of the given width), in the
    reference's operation order (CellModel.derive)."""

    name = 'globals_deriver'
    defaults = {'width': 1, 'initial_mass': 1339.0, 'periplasm_volume_fraction': 0.3, 'density': 1100.0}

    def __init__(self, initial_parameters=None):
        super().__init__(initial_parameters)
        from lens_amd.cells import CellModel
        p = self.parameters
        self.model = CellModel(width=p['width'], density=p['density'], avogadro=AVOGADRO)
        self._models = {(p['width'], p['density']): self.model}

    def is_deriver(self):
        return True

    def _model(self, width, density):
        # derive_globals.py:133-135 reads width and density from the store on every
        # call: one CellModel per (width, density) pair seen
        key = (width, density)
        m = self._models.get(key)
        if m is None:
            from lens_amd.cells import CellModel
            m = self._models[key] = CellModel(width=width, density=density, avogadro=AVOGADRO)
        return m

    def _derived(self, mass, width=None, density=None):
        p = self.parameters
        model = self._model(p['width'] if width is None else width, p['density'] if density is None else density)
        volume, m2c, length, area = model.derive(mass)
        return {'volume': volume, 'mmol_to_counts': m2c, 'length': length, 'surface_area': area,
                'periplasm_volume': volume * self.parameters['periplasm_volume_fraction']}

    def ports_schema(self):
        mass = self.parameters['initial_mass']
        d = self._derived(mass)
        default = {'mass': mass, 'volume': d['volume'], 'mmol_to_counts': d['mmol_to_counts'],
                   'density': self.parameters['density'], 'width': self.parameters['width'],
                   'length': d['length'], 'surface_area': d['surface_area'],
                   'periplasm_volume': d['periplasm_volume']}
        set_states = ('volume', 'mmol_to_counts', 'length', 'surface_area', 'periplasm_volume')
        split = ('volume', 'length', 'surface_area', 'periplasm_volume')
        emit = ('volume', 'width', 'length', 'surface_area')
        schema = {}
        for k, v in default.items():
            s = {'_default': v}
            if k in set_states:
                s['_updater'] = 'set'
            if k in emit:
                s['_emit'] = True
            if k in split:
                s['_divider'] = 'split'
            schema[k] = s
        return {'global': schema}

    def next_update(self, timestep, states):
        g = states['global']
        return {'global': self._derived(g['mass'], g.get('width'), g.get('density'))}


def growth_division_minimal(agent_id, growth_rate=0.000275, boundary_path=('boundary',)):
    """The growth_division_minimal compartment of one agent: processes and
    topology, derivers first (process.py:179-182 merges them in front)."""
    growth = GrowthProtein({'growth_rate': growth_rate})
    return {
        'processes': {
            'mass_deriver': TreeMass({'mw_paths': {('internal', 'protein'): growth.parameters['protein_mw']}}),
            'global_deriver': DeriveGlobals(),
            'growth': growth,
            'division': MetaDivision({'agent_id': agent_id, 'daughter_path': (),
                                      'compartment': lambda cfg: growth_division_minimal(
                                          cfg['agent_id'], growth_rate, boundary_path)})},
        'topology': {
            'mass_deriver': {'global': boundary_path, 'agent': ()},
            'global_deriver': {'global': boundary_path},
            'growth': {'internal': ('internal',), 'global': boundary_path},
            'division': {'global': boundary_path, 'cells': ('..', '..', 'agents')}}}
