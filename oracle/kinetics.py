"""Oracle (TEST INFRASTRUCTURE ONLY): per-agent convenience-kinetics step,
exchange, non-spatial environment, C1 replay and the ODE (odeint) oracle.

Restates, agent by agent in plain Python/numpy:
  * ConvenienceKinetics.next_update ........ vivarium/processes/convenience_kinetics.py:303-352
  * update_field_with_exchange ............. vivarium/core/registry.py:149-183
  * get_bin_site / get_bin_volume .......... vivarium/library/lattice_utils.py:18-58
  * NonSpatialEnvironment (field[0][0] -> external, depth = V/1um^2)
                                            vivarium/processes/nonspatial_environment.py:22-82
  * DeriveGlobals volume / mmol_to_counts .. vivarium/processes/derive_globals.py:213-234
  * process_in_experiment / Experiment.update step order for one agent
                                            vivarium/core/composition.py:225-279,
                                            vivarium/core/experiment.py:1351-1450
The convenience_kinetics.csv fixture was produced with scipy<1.4's Avogadro
constant (SURVEY.md §0 finding 2), so N_A is a parameter here.
"""

from __future__ import annotations

import math

import numpy as np

from oracle.rate_laws import OracleFluxModel

N_A_LEGACY = 6.022140857e23   # CODATA 2014 (scipy < 1.4): the fixture's constant
N_A_CODATA2018 = 6.02214076e23

PORT_IDS = ('internal', 'external', 'fluxes', 'fields', 'global')


def mmol_to_counts(mass_fg=1339.0, density_g_per_L=1100.0, avogadro=N_A_LEGACY):
    """(N_A/mol * mass/density).to('L/mmol') (derive_globals.py:219-220)."""
    volume_L = mass_fg / density_g_per_L * 1e-15
    return avogadro * volume_L * 1e-3


def bin_site(location, n_bins, bounds):
    """floor(loc*n/bound) % n on both axes (lattice_utils.py:34-40)."""
    i = int(math.floor(location[0] * n_bins[0] / bounds[0])) % n_bins[0]
    j = int(math.floor(location[1] * n_bins[1] / bounds[1])) % n_bins[1]
    return i, j


def bin_volume_L(n_bins, bounds, depth):
    """(depth*bx*by)*1e-15 / (nx*ny) litres (lattice_utils.py:57-58)."""
    return (depth * bounds[0] * bounds[1]) * 1e-15 / (n_bins[0] * n_bins[1])


def count_to_mM(count, bin_volume, avogadro=N_A_LEGACY):
    """count / (bin_volume*N_A) mol/L -> mmol/L (lattice_utils.py:73, registry.py:180-182)."""
    return count / (bin_volume * avogadro) * 1000.0


class OracleAgent:
    """One ConvenienceKinetics agent, evaluated exactly as the reference does."""

    def __init__(self, reactions, kinetic_parameters, port_ids=PORT_IDS):
        self.reactions = reactions
        self.model = OracleFluxModel(reactions, kinetic_parameters)
        self.port_ids = list(port_ids)

    def next_update(self, timestep, states, m2c):
        """Returns (fluxes dict, {port: {state: delta}}, {mol: int count})."""
        flat = {}
        for port, sd in states.items():
            if sd:
                for k, v in sd.items():
                    flat[(port, k)] = v
        fluxes = self.model.get_fluxes(flat)
        deltas = {p: {} for p in self.port_ids}
        counts = {}
        for rid, flux in fluxes.items():
            for port_state, coeff in self.reactions[rid]['stoichiometry'].items():
                for port in self.port_ids:
                    if port in port_state:
                        name = port_state[1]
                        sflux = coeff * flux * timestep
                        if port == 'external':
                            counts[name] = counts.get(name, 0) + int(sflux * m2c)
                        else:
                            deltas[port][name] = deltas[port].get(name, 0) + sflux
        return fluxes, deltas, counts


def replay_single_agent(reactions, kinetic_parameters, initial_state, n_steps,
                        timestep=1.0, env_volume_L=1e-14, mass_fg=1339.0,
                        avogadro=N_A_LEGACY, field_init=1.0):
    """C1: process_in_experiment with a NonSpatialEnvironment (one agent).

    Order per step (experiment.py:1365-1446): the process computes from the
    step-start state; the update is applied (internal accumulate, field
    exchange); derivers then run (NonSpatialEnvironment sets external :=
    field[0][0]).  At t=0 the derivers ran once, so external starts at the
    field's initial value (1.0, nonspatial_environment.py:40-44), not at the
    configured initial_state external values.
    Returns list of {'internal': {...}, 'external': {...}} per emitted time.
    """
    agent = OracleAgent(reactions, kinetic_parameters)
    internal = dict(initial_state.get('internal', {}))
    fields = {m: field_init for m in initial_state.get('external', {})}
    external = dict(fields)
    m2c = mmol_to_counts(mass_fg, avogadro=avogadro)
    # NonSpatialEnvironment: depth = V / (1um*1um) in um; bin volume = depth*1*1*1e-15/1
    depth_um = env_volume_L * 1e15
    bvol = bin_volume_L([1, 1], [1.0, 1.0], depth_um)
    out = [{'internal': dict(internal), 'external': dict(external)}]
    for _ in range(n_steps):
        _, deltas, counts = agent.next_update(
            timestep, {'internal': internal, 'external': external}, m2c)
        for k, d in deltas['internal'].items():
            internal[k] = internal[k] + d
        for mol, c in counts.items():
            fields[mol] = fields[mol] + count_to_mM(c, bvol, avogadro)
        external = dict(fields)
        out.append({'internal': dict(internal), 'external': dict(external)})
    return out


# ---------------------------------------------------------------------------
# ODE oracle: the augmented right-hand side integrated by scipy odeint
# ---------------------------------------------------------------------------

class OracleODE:
    """d(internal)/dt = sum_r coeff*flux_r (non-external ports), d(acc_r)/dt = flux_r.

    External species (and enzymes) are held at their step-start values; the
    exchange over the step is int(coeff * acc_r * mmol_to_counts), the ODE
    analogue of convenience_kinetics.py:327-331 (acc_r replaces flux*timestep),
    the same accumulator construction the reference's only odeint path uses
    (Kremling2007_transport.py:386-405).
    """

    def __init__(self, reactions, kinetic_parameters, port_ids=PORT_IDS):
        self.agent = OracleAgent(reactions, kinetic_parameters, port_ids)
        self.rids = self.agent.model.reaction_ids
        # dynamic keys in encounter order
        self.dyn = []
        for rid in self.rids:
            for port_state in reactions[rid]['stoichiometry']:
                for port in port_ids:
                    if port in port_state and port != 'external':
                        key = (port, port_state[1])
                        if key not in self.dyn:
                            self.dyn.append(key)

    def rhs(self, y, conc_fixed):
        conc = dict(conc_fixed)
        for i, key in enumerate(self.dyn):
            conc[key] = y[i]
        fluxes = self.agent.model.get_fluxes(conc)
        dy = np.zeros(len(self.dyn) + len(self.rids))
        acc = {}
        for rid in self.rids:
            f = fluxes[rid]
            for port_state, coeff in self.agent.reactions[rid]['stoichiometry'].items():
                for port in self.agent.port_ids:
                    if port in port_state and port != 'external':
                        key = (port, port_state[1])
                        acc[key] = acc.get(key, 0) + coeff * f
        for i, key in enumerate(self.dyn):
            dy[i] = acc.get(key, 0.0)
        for r, rid in enumerate(self.rids):
            dy[len(self.dyn) + r] = fluxes[rid]
        return dy

    def integrate(self, conc, timestep, rtol=1e-12, atol=1e-15, t_eval=None):
        from scipy.integrate import odeint
        y0 = np.array([conc[k] for k in self.dyn] + [0.0] * len(self.rids), dtype=np.float64)
        ts = np.array([0.0, timestep]) if t_eval is None else t_eval
        sol, info = odeint(lambda y, t: self.rhs(y, conc), y0, ts, rtol=rtol, atol=atol,
                           full_output=True, mxstep=100000)
        return sol[-1], info

    def step(self, conc, timestep, m2c, rtol=1e-12, atol=1e-15):
        """Returns (new dyn values dict, mean fluxes dict, counts dict)."""
        y, _ = self.integrate(conc, timestep, rtol, atol)
        nd = len(self.dyn)
        new = {k: y[i] for i, k in enumerate(self.dyn)}
        fluxes = {rid: y[nd + r] / timestep for r, rid in enumerate(self.rids)}
        counts = {}
        for r, rid in enumerate(self.rids):
            for port_state, coeff in self.agent.reactions[rid]['stoichiometry'].items():
                if 'external' in port_state:
                    name = port_state[1]
                    counts[name] = counts.get(name, 0) + int(coeff * y[nd + r] * m2c)
        return new, fluxes, counts


def params_dict(param_names, config, pvec):
    """Per-agent parameter vector (RateLawTable.param_names order) -> a
    reference ``kinetic_parameters`` dict ({rxn: {enzyme: {mol: Km, 'kcat_f':
    kcat}}}); ``None`` Kms of the configuration are kept (they are not table
    parameters)."""
    kp = {}
    for (kind, rid, enz, *mol), v in zip(param_names, pvec):
        kp.setdefault(rid, {}).setdefault(enz, {})
        kp[rid][enz]['kcat_f' if kind == 'kcat' else mol[0]] = float(v)
    for rid in config['kinetic_parameters']:
        for enz, p in config['kinetic_parameters'][rid].items():
            for k, v in p.items():
                if v is None:
                    kp[rid][enz][k] = None
    return kp
