"""Rate-law compiler: convenience-kinetics reaction dicts -> flat SoA reaction table.

This is the host half of the drop-in boundary.  It takes exactly the
``reactions`` / ``kinetic_parameters`` dictionaries a reference
``ConvenienceKinetics`` process is configured with and produces the flat,
index-only description the HIP kernels walk (``include/vk_kinetics.h``,
``vk_table_desc``).  Per-agent numbers (kcat, Km) are *not* baked into the
table: they become parameter slots, so one table serves a whole colony of
agents with heterogeneous parameters (SoA ``params[slot][agent]``).

Semantics restated (not copied) from the reference:

* ``make_configuration`` (vivarium/library/kinetic_rate_laws.py:43-98):
  per enzyme, the partition is the reactant sets of every *other* reaction
  that enzyme catalyses followed by this reaction's own cofactor sets
  (forward reactants, plus products when ``is reversible``).  The partition
  entry is overwritten per reaction, so the last reaction processed for an
  enzyme decides it (:95), and that list *shares list objects* with the
  last reaction's cofactor sets.
* ``construct_convenience_rate_law`` (:106-180): molecules whose parameter
  value is ``None`` are removed *in place* from the shared partition lists
  and from the rate law's cofactor lists (:127-135).  Because the closures
  read those lists lazily, every rate law sees the lists as they stand after
  *all* rate laws were built -- the aliasing quirk.  We replay the removals
  on real Python lists with the same object sharing and flatten afterwards.
  A truthy ``kcat_r`` makes the reference raise ``NameError`` (:139-140);
  we raise the same.
* ``KineticFluxModel.get_fluxes`` (:277-297): flux[r] = 0.0 + sum over the
  reaction's enzymes (``catalyzed by`` order, enzymes without parameters
  skipped as in ``make_rate_laws`` :219-222); reaction order is the key
  order of ``kinetic_parameters`` (:265).
* ``ConvenienceKinetics.next_update`` (vivarium/processes/convenience_kinetics.py:320-349):
  the per-(reaction, stoichiometry entry) loop over ``port_ids`` with the
  tuple-membership test ``port_id in port_state_id`` (:323-326).  Entries
  matching ``'external'`` become integer exchange counts, entries matching
  any other port accumulate into that port's state; the encounter order is
  kept so device sums are bit-identical to the reference's Python sums.
"""

from __future__ import annotations

import dataclasses
from typing import Any, Dict, List, Sequence, Tuple

import numpy as np

# ports the reference ConvenienceKinetics exposes (convenience_kinetics.py:218-227, :235)
DEFAULT_PORT_IDS = ('internal', 'external', 'fluxes', 'fields', 'global')

PARAM_KCAT = 0
PARAM_KM = 1


@dataclasses.dataclass
class RateLawTable:
    """Flat, index-only reaction table (one per network, shared by all agents).

    Arrays are int32 / float64 numpy arrays laid out exactly as the C-ABI
    ``vk_table_desc`` expects.
    """

    species: List[Tuple[str, str]]      # species keys (port, name); index = SoA row
    n_dyn: int                          # species[:n_dyn] receive per-step deltas
    reaction_ids: List[str]             # flux order (kinetic_parameters key order)
    external_ids: List[str]             # molecules receiving exchange counts
    param_names: List[Tuple]            # ('kcat', rxn, enzyme) | ('km', rxn, enzyme, mol)
    param_defaults: np.ndarray          # float64 [n_params] values from the config
    rate_laws: List[Tuple[str, Tuple]]  # (reaction_id, enzyme) per rate law, eval order
    # rate laws (eval order == get_fluxes order)
    rl_reaction: np.ndarray
    rl_enzyme: np.ndarray
    rl_kcat: np.ndarray
    rl_num_ptr: np.ndarray              # [L+1] -> set index (numerator cofactor sets)
    rl_den_ptr: np.ndarray              # [L+1] -> set index (partition sets)
    set_ptr: np.ndarray                 # [n_sets+1] -> member index
    mem_species: np.ndarray             # [M] species index
    mem_param: np.ndarray               # [M] Km parameter slot
    # internal (accumulate) updates, CSR by dyn species, reference encounter order
    upd_ptr: np.ndarray
    upd_rxn: np.ndarray
    upd_coeff: np.ndarray
    # exchange counts, CSR by external molecule
    ex_ptr: np.ndarray
    ex_rxn: np.ndarray
    ex_coeff: np.ndarray

    @property
    def n_species(self) -> int:
        return len(self.species)

    @property
    def n_reactions(self) -> int:
        return len(self.reaction_ids)

    @property
    def n_rate_laws(self) -> int:
        return len(self.rl_reaction)

    @property
    def n_params(self) -> int:
        return len(self.param_names)

    @property
    def n_ext(self) -> int:
        return len(self.external_ids)

    def species_index(self, key) -> int:
        return self.species.index(tuple(key))

    def flops_rhs(self) -> int:
        """Algorithmic FP64 flops of one right-hand-side evaluation.

        Counted as the kernels execute them (a divide counts 1):
        numerator set of k members: k (c*invKm) + (k-1) products + 1 (kcat*) + 1 (sum);
        x enzyme: 1; partition set of k members: k (c*invKm) + k (1+) + (k-1)
        products + 1 (-1) + 1 (sum); num/den: 1; reaction sum: 1;
        each stoichiometry entry: 2 (coeff*flux, +=).
        """
        f = 0
        for l in range(self.n_rate_laws):
            for s in range(self.rl_num_ptr[l], self.rl_num_ptr[l + 1]):
                k = int(self.set_ptr[s + 1] - self.set_ptr[s])
                f += k + max(k - 1, 0) + 2
            f += 1
            for s in range(self.rl_den_ptr[l], self.rl_den_ptr[l + 1]):
                k = int(self.set_ptr[s + 1] - self.set_ptr[s])
                f += 2 * k + max(k - 1, 0) + 2
            f += 2
        f += 2 * len(self.upd_rxn)
        return f

    def arrays(self) -> Dict[str, np.ndarray]:
        return {k: getattr(self, k) for k in (
            'rl_reaction', 'rl_enzyme', 'rl_kcat', 'rl_num_ptr', 'rl_den_ptr',
            'set_ptr', 'mem_species', 'mem_param', 'upd_ptr', 'upd_rxn',
            'upd_coeff', 'ex_ptr', 'ex_rxn', 'ex_coeff')}


def _reactants(stoich) -> list:
    return [mol for mol, coeff in stoich.items() if coeff < 0]


def _products(stoich) -> list:
    return [mol for mol, coeff in stoich.items() if coeff > 0]


def _configure(reactions: Dict[str, Any]):
    """Per-enzyme partition + per-(enzyme, reaction) cofactor sets, with the
    reference's list-object sharing (kinetic_rate_laws.py:43-98)."""
    config: Dict[Any, Dict[str, Any]] = {}
    for rid, spec in reactions.items():
        for enz in spec['catalyzed by']:
            config.setdefault(enz, {'partition': [], 'cofactors': {}})
    for rid, spec in reactions.items():
        stoich = spec.get('stoichiometry')
        sets = [_reactants(stoich)]
        if spec.get('is reversible', False):
            sets.append(_products(stoich))
        for enz in spec.get('catalyzed by', None):
            rivals = [_reactants(reactions[other]['stoichiometry'])
                      for other, spec2 in reactions.items()
                      if other != rid and enz in spec2['catalyzed by']]
            # rivals are fresh lists; `sets` are shared with cofactors[rid]
            config[enz]['partition'] = rivals + sets
            config[enz]['cofactors'][rid] = sets
    return config


def compile_rate_laws(reactions: Dict[str, Any],
                      kinetic_parameters: Dict[str, Any],
                      port_ids: Sequence[str] = DEFAULT_PORT_IDS) -> RateLawTable:
    """Compile a ConvenienceKinetics network into a :class:`RateLawTable`."""
    reaction_ids = list(kinetic_parameters.keys())
    for rid in reactions:
        if rid not in kinetic_parameters:
            # make_rate_laws indexes kinetic_parameters[reaction_id] (kinetic_rate_laws.py:220)
            raise KeyError(rid)
    for rid in reaction_ids:
        if rid not in reactions:
            # next_update indexes self.reactions[reaction_id] (convenience_kinetics.py:321)
            raise KeyError(rid)

    config = _configure(reactions)

    # Build rate laws in make_rate_laws order, performing the in-place None
    # removals as each is constructed (kinetic_rate_laws.py:212-235, :127-135).
    built = []  # (rid, enzyme, cofactor_sets(list objs), partition(list obj), params)
    for rid, spec in reactions.items():
        for enz in spec.get('catalyzed by'):
            if enz not in kinetic_parameters[rid]:
                continue
            params = kinetic_parameters[rid][enz]
            sets = config[enz]['cofactors'][rid]
            partition = config[enz]['partition']
            for pname, pval in params.items():
                if 'kcat' in pname or pval is not None:
                    continue
                for part in partition:
                    if pname in part:
                        part.remove(pname)
                for cset in sets:
                    if pname in cset:
                        cset.remove(pname)
            if params.get('kcat_r'):
                raise NameError(
                    "name 'cofactors' is not defined (reference kinetic_rate_laws.py:140 "
                    "raises for any truthy kcat_r; reaction %r, enzyme %r)" % (rid, enz))
            built.append((rid, enz, sets, partition, params))

    # ---- species indexing: updated (non-external) species first -------------
    upd_entries: Dict[Tuple[str, str], List[Tuple[int, float]]] = {}
    ex_entries: Dict[str, List[Tuple[int, float]]] = {}
    for r, rid in enumerate(reaction_ids):
        for port_state, coeff in reactions[rid]['stoichiometry'].items():
            for port in port_ids:
                if port in port_state:
                    name = port_state[1]
                    if port == 'external':
                        ex_entries.setdefault(name, []).append((r, float(coeff)))
                    else:
                        upd_entries.setdefault((port, name), []).append((r, float(coeff)))

    species: List[Tuple[str, str]] = list(upd_entries.keys())
    n_dyn = len(species)
    index: Dict[Tuple, int] = {k: i for i, k in enumerate(species)}

    def sidx(key) -> int:
        key = tuple(key)
        if key not in index:
            index[key] = len(species)
            species.append(key)
        return index[key]

    # ---- parameter slots + flattened sets ------------------------------------
    param_names: List[Tuple] = []
    param_vals: List[float] = []
    slot_of: Dict[Tuple, int] = {}

    def pslot(name: Tuple, value) -> int:
        if name not in slot_of:
            slot_of[name] = len(param_names)
            param_names.append(name)
            param_vals.append(float(value))
        return slot_of[name]

    rl_reaction, rl_enzyme, rl_kcat = [], [], []
    rl_num_ptr, rl_den_ptr = [0], [0]
    set_ptr = [0]
    mem_species, mem_param = [], []
    rate_laws = []
    for rid, enz, sets, partition, params in built:
        kcat = params.get('kcat_f')
        if kcat is None:
            raise TypeError('rate law %r/%r has no kcat_f (reference multiplies None, '
                            'kinetic_rate_laws.py:162)' % (rid, enz))
        rate_laws.append((rid, enz))
        rl_reaction.append(reaction_ids.index(rid))
        rl_enzyme.append(sidx(enz))
        rl_kcat.append(pslot(('kcat', rid, enz), kcat))

    # Flatten after every removal has happened (lazy closure semantics).
    # Numerator sets of all rate laws first, then all partition sets.
    def flatten(groups_of, ptr):
        for rid, enz, sets, partition, params in built:
            for members in groups_of(sets, partition):
                for mol in members:
                    if mol not in params:
                        # rate_law looks up parameters[molecule] (kinetic_rate_laws.py:160,173)
                        raise KeyError(mol)
                    mem_species.append(sidx(mol))
                    mem_param.append(pslot(('km', rid, enz, mol), params[mol]))
                set_ptr.append(len(mem_species))
            ptr.append(len(set_ptr) - 1)

    flatten(lambda sets, partition: sets, rl_num_ptr)
    rl_den_ptr[0] = len(set_ptr) - 1
    flatten(lambda sets, partition: partition, rl_den_ptr)

    # ---- update / exchange CSR -------------------------------------------------
    upd_ptr, upd_rxn, upd_coeff = [0], [], []
    for key in species[:n_dyn]:
        for r, c in upd_entries[key]:
            upd_rxn.append(r)
            upd_coeff.append(c)
        upd_ptr.append(len(upd_rxn))
    external_ids = list(ex_entries.keys())
    ex_ptr, ex_rxn, ex_coeff = [0], [], []
    for name in external_ids:
        for r, c in ex_entries[name]:
            ex_rxn.append(r)
            ex_coeff.append(c)
        ex_ptr.append(len(ex_rxn))

    i32 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.int32))
    f64 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return RateLawTable(
        species=species, n_dyn=n_dyn, reaction_ids=reaction_ids,
        external_ids=external_ids, param_names=param_names,
        param_defaults=f64(param_vals), rate_laws=rate_laws,
        rl_reaction=i32(rl_reaction), rl_enzyme=i32(rl_enzyme), rl_kcat=i32(rl_kcat),
        rl_num_ptr=i32(rl_num_ptr), rl_den_ptr=i32(rl_den_ptr), set_ptr=i32(set_ptr),
        mem_species=i32(mem_species), mem_param=i32(mem_param),
        upd_ptr=i32(upd_ptr), upd_rxn=i32(upd_rxn), upd_coeff=f64(upd_coeff),
        ex_ptr=i32(ex_ptr), ex_rxn=i32(ex_rxn), ex_coeff=f64(ex_coeff))
