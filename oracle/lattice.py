"""Oracle (TEST INFRASTRUCTURE ONLY): diffusion_field lattice + agent coupling.

Restates:
  * DiffusionField coefficient D/(dx*dy) ........ vivarium/processes/diffusion_field.py:251-260
  * diffusion_delta sub-stepping ................. :385-394 (t += dt while t < timestep)
  * convolve(f, LAPLACIAN_2D, mode='reflect') .... :35, :391 -- summation order
    up, left, centre(-4), right, down (row = axis 0), bit-identical to scipy
    (pinned by tests/golden/stencil.npz)
  * uniform-field skip ........................... :396-407
  * local environments (pre-step field at bin) ... :362-379
  * exchange updater (agent order) ............... vivarium/core/registry.py:149-183
  * lattice step order: all processes compute from the
    step-start state; the diffusion delta lands first, then each agent's
    exchange in agent order; external := pre-step field at the bin.
"""

from __future__ import annotations

import numpy as np

from oracle.kinetics import bin_site, bin_volume_L, count_to_mM, N_A_LEGACY


def n_substeps(timestep, dt_max=0.01):
    t, dt, n = 0.0, min(timestep, dt_max), 0
    while t < timestep:
        t += dt
        n += 1
    return n


def laplacian_reflect(f):
    p = np.pad(f, 1, mode='edge')
    up, down = p[:-2, 1:-1], p[2:, 1:-1]
    left, right = p[1:-1, :-2], p[1:-1, 2:]
    centre = p[1:-1, 1:-1]
    return (((up + left) + (-4.0 * centre)) + right) + down


def diffuse(field, timestep, diffusion, n_bins, bounds, dt_max=0.01):
    """Returns the new field (field + delta, as the accumulate updater applies it)."""
    if len(np.unique(field)) == 1:
        return field + np.zeros_like(field)
    dx = bounds[0] / n_bins[0]
    dy = bounds[1] / n_bins[1]
    coef = diffusion / (dx * dy)
    fn = field.copy()
    sub = min(timestep, dt_max)
    for _ in range(n_substeps(timestep, dt_max)):
        fn += coef * sub * laplacian_reflect(fn)
    return field + (fn - field)


def lattice_step(fields, agents_loc, counts, n_bins, bounds, depth, timestep, diffusion,
                 avogadro=N_A_LEGACY):
    """One lattice step for the environment side.

    fields: {mol: ndarray}; agents_loc: [(x, y)] in agent order;
    counts: {mol: [int per agent]} exchange counts computed this step.
    Returns (new fields, local environments {mol: [value per agent]} from the
    pre-step fields).
    """
    bvol = bin_volume_L(n_bins, bounds, depth)
    sites = [bin_site(loc, n_bins, bounds) for loc in agents_loc]
    local = {m: np.array([f[s] for s in sites]) for m, f in fields.items()}
    new = {m: diffuse(f, timestep, diffusion, n_bins, bounds) for m, f in fields.items()}
    for m, per_agent in counts.items():
        if m not in new:
            continue
        f = new[m]
        for a, c in enumerate(per_agent):
            i, j = sites[a]
            f[i, j] = f[i, j] + count_to_mM(c, bvol, avogadro)
    return new, local


def diffusion_delta(field, timestep, diffusion, n_bins, bounds, dt_max=0.01):
    """DiffusionField.diffuse for one field (diffusion_field.py:385-407): the delta
    field_new - field, zeros for a uniform field."""
    if len(np.unique(field)) == 1:
        return np.zeros_like(field)
    dx = bounds[0] / n_bins[0]
    dy = bounds[1] / n_bins[1]
    coef = diffusion / (dx * dy)
    fn = field.copy()
    sub = min(timestep, dt_max)
    t = 0.0
    while t < timestep:
        fn += coef * sub * laplacian_reflect(fn)
        t += sub
    return fn - field
