"""Generate tests/golden/{c2,c3kin}_odeint_traj.npz (TEST FIXTURE GENERATOR).

c2: BASELINE config 2: 10,000 heterogeneous glc_lct agents,
external concentrations held per agent, Delta t = 1 s, 100 steps; a sample of
304 agents (every 33rd).  glc_lct's fluxes do not depend on its integrated
species (pep_c has no Km), so its ODE is exactly solvable by any RK method.
c3kin: the kinetics of BASELINE configs 3-4 (glc_ac: acetate secretion runs
on g6p_c, so the ODE is genuinely non-linear) in the same held-externals
setting: 100,000 agents, a sample of 301 (every 333rd).

For each sampled agent this integrates the restated ODE right-hand
side (oracle.kinetics.OracleODE: the reference rate laws of
kinetic_rate_laws.py:149-178 plus flux integrals, the accumulator
construction of Kremling2007_transport.py:386-405) with scipy's odeint
(LSODA, rtol 1e-12, atol 1e-15), restarted at every step from the previous
step's end state -- the reference's odeint call pattern
(Kremling2007_transport.py:354-384) -- and records the dynamic species and
mean fluxes after every 10th step.

    python tests/golden/make_odeint_traj.py [c2 c3kin c5kin]

c5kin: the C5 network (50 species, 40 reactions, 10 enzymes; stiff), 4096
agents with lognormal(0, 0.2) parameters, a sample of 64 (every 64th),
every one of 10 one-second steps.
"""

from __future__ import annotations

import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from lens_amd import configs  # noqa: E402
from lens_amd.rate_law_compiler import compile_rate_laws  # noqa: E402
from oracle.kinetics import OracleODE, mmol_to_counts, params_dict  # noqa: E402

CASES = {  # name: (network, agents, stride, lognormal sigma, steps, record every)
    'c2': (configs.glc_lct_config, 10_000, 33, 0.25, 100, 10),
    'c3kin': (configs.glc_ac_config, 100_000, 333, 0.25, 100, 10),
    'c5kin': (lambda: configs.synthetic_network(n_species=50, n_reactions=40, n_enzymes=10),
              4096, 64, 0.2, 10, 1),
}


def _setup(name):
    make, n_agents, _, sigma, _, _ = CASES[name]
    cfg = make()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    params, conc = configs.heterogeneous_colony(t, cfg, n_agents, seed=configs.SEED, sigma=sigma)
    return cfg, t, params, conc


def _one(job):
    name, a = job
    cfg, t, params, conc = _setup(name)
    STEPS, EVERY = CASES[name][4:]
    ode = OracleODE(cfg['reactions'], params_dict(t.param_names, cfg, params[:, a]))
    c = {k: conc[s, a] for s, k in enumerate(t.species)}
    ys, fs = [], []
    for step in range(1, STEPS + 1):
        new, fl, _ = ode.step(c, 1.0, mmol_to_counts())
        c.update(new)
        if step % EVERY == 0:
            ys.append([c[t.species[s]] for s in range(t.n_dyn)])
            fs.append([fl[r] for r in t.reaction_ids])
    return a, ys, fs


def main():
    for name in sys.argv[1:] or sorted(CASES):
        cfg, t, params, conc = _setup(name)
        _, n_agents, stride, _, steps, every = CASES[name]
        sample = np.arange(0, n_agents, stride)
        with Pool(min(8, os.cpu_count() or 1)) as pool:
            res = sorted(pool.map(_one, [(name, int(a)) for a in sample]))
        y = np.array([r[1] for r in res])          # [agent, checkpoint, n_dyn]
        f = np.array([r[2] for r in res])          # [agent, checkpoint, n_reactions]
        np.savez_compressed(os.path.join(HERE, '%s_odeint_traj.npz' % name), sample=sample, y=y, flux=f,
                            params=params[:, sample], conc=conc[:, sample],
                            steps=np.arange(every, steps + 1, every), m2c=mmol_to_counts())
        print('wrote', name, y.shape)


if __name__ == '__main__':
    main()
