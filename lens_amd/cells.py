"""Cell growth, derivers and division for a device-resident colony.

Host half of ``vk_cell_step`` / ``vk_divide_*`` (include/vk_kinetics.h).  A
:class:`CellModel` carries the reference processes' parameters:

``model='growth_protein'`` -- GrowthProtein + TreeMass + DeriveGlobals +
    MetaDivision (the ``growth_division_minimal`` agent of the reference's
    colony_metrics experiment; vivarium/compartments/growth_division_minimal.py).
``model='growth'`` -- Growth + DeriveGlobals + DivisionVolume + MetaDivision
    (SURVEY §8d C5).

Scalars that the reference computes with numpy / pint (``exp(r*dt)``, the
capsule constants, unit-conversion factors) are evaluated here, in Python,
exactly as the reference writes them, and handed to the kernel, so the
device arithmetic reproduces the reference bit for bit.

Random remainder of GrowthProtein (growth_protein.py:94-96):
``rng='stream'`` draws the uniforms on the host from numpy's MT19937 in
agent order -- the reference's own stream (``np.random.seed(seed)``; the
reference's colony_metrics setup consumes ``setup_draws=2`` draws first);
``rng='philox'`` draws them on the device from Philox4x32-10 keyed by
(seed, step, lineage), independent of agent order and rank count.
"""

from __future__ import annotations

import ctypes
import dataclasses
import math

import numpy as np

from lens_amd import native

N_A_LEGACY = 6.022140857e23
PI = math.pi
# unit-conversion factors as pint evaluates them in the reference
FG_PER_G = 1 / 1e-15                          # g -> fg (TreeMass.calculate_mass)
VOLUME_TO_FL = 1e-18 / 1e-3 * 1e18 * 1e-3     # fg*L/g -> fL (DeriveGlobals volume.to('fL'))

MODELS = {'growth_protein': native.VK_GROWTH_PROTEIN, 'growth': native.VK_GROWTH_MASS}
RNGS = {'stream': native.VK_RNG_STREAM, 'philox': native.VK_RNG_PHILOX}


@dataclasses.dataclass
class CellModel:
    model: str = 'growth_protein'
    growth_rate: float = 0.000275          # growth_protein.py:27 (Growth: 0.0006, growth.py:61)
    division_volume: float = 2.4           # fL, division_volume.py:13
    initial_mass: float = 1339.0           # fg
    protein_mw: float = 2.09e4             # g/mol, growth_protein.py:26
    width: float = 1                       # um, derive_globals.py:60 (an int there: emitted as 1)
    density: float = 1100.0                # g/L, derive_globals.py:93
    avogadro: float = N_A_LEGACY
    rng: str = 'stream'
    seed: int = 1
    setup_draws: int = 0

    def __post_init__(self):
        if self.model not in MODELS:
            raise ValueError('model must be one of %s' % sorted(MODELS))
        if self.rng not in RNGS:
            raise ValueError('rng must be one of %s' % sorted(RNGS))
        self._rs = None

    # -- reference formulas (Python floats, the reference's operation order) --
    def initial_protein(self) -> float:
        """growth_protein.py:46-47: initial_mass.to('g') / protein_mw * N_A."""
        return self.initial_mass * 1e-15 / self.protein_mw * self.avogadro

    def tree_mass(self, protein: float) -> float:
        return 0.0 + (self.protein_mw * (protein / self.avogadro)) * FG_PER_G

    def capsule(self):
        radius = self.width / 2
        return {'cap_volume': (4 / 3) * PI * radius ** 3, 'cap_area': PI * radius ** 2,
                'two_r': 2 * radius, 'sa_const': 3 * PI * radius ** 2, 'sa_lin': 2 * PI * radius}

    def derive(self, mass: float):
        """DeriveGlobals on one mass: (volume fL, mmol_to_counts, length, surface_area)."""
        c = self.capsule()
        raw = mass / self.density
        length = (raw - c['cap_volume']) / c['cap_area'] + c['two_r']
        area = c['sa_const'] + c['sa_lin'] * (length - self.width)
        return raw * VOLUME_TO_FL, self.avogadro * (raw * 1e-15) * 1e-3, length, area

    def initial_rows(self, n: int, mass=None):
        """Cell rows [VK_CELL_ROWS, n] + mmol_to_counts [n] after the
        initial deriver pass (experiment.py:1247)."""
        rows = np.zeros((native.VK_CELL_ROWS, n))
        m2c = np.zeros(n)
        if self.model == 'growth_protein':
            p0 = self.initial_protein()
            mass = np.full(n, self.tree_mass(p0))
            rows[native.VK_CELL_PROTEIN] = p0
        else:
            mass = np.full(n, self.initial_mass) if mass is None else np.asarray(mass, dtype=np.float64)
        for a in range(n):
            v, mc, length, area = self.derive(float(mass[a]))
            rows[:4, a] = (mass[a], v, length, area)
            m2c[a] = mc
        return rows, m2c

    # -- kernel parameters ----------------------------------------------------
    def vk_params(self, dt: float, step: int) -> native.VkCellParams:
        p = native.VkCellParams()
        p.model = MODELS[self.model]
        p.rng = RNGS[self.rng]
        p.factor = float(np.exp(self.growth_rate * dt))
        p.divide_protein = self.initial_protein() * 2
        p.division_volume = self.division_volume
        p.protein_mw = self.protein_mw
        p.avogadro = self.avogadro
        p.fg_per_g = FG_PER_G
        p.density = self.density
        p.volume_to_fl = VOLUME_TO_FL
        for k, v in self.capsule().items():
            setattr(p, k, v)
        p.width = self.width
        p.seed = int(self.seed) & (2 ** 64 - 1)
        p.step = int(step) & (2 ** 64 - 1)
        return p

    def host_uniforms(self, n: int) -> np.ndarray:
        """The next n draws of numpy's MT19937 stream (rng='stream')."""
        if self._rs is None:
            self._rs = np.random.RandomState(self.seed)
            if self.setup_draws:
                self._rs.random_sample(self.setup_draws)
        return self._rs.random_sample(n)


def lineage_ids(roots, root, depth, path):
    """Phylogeny id strings (meta_division.py:15-18) from the lineage arrays."""
    out = []
    for r, d, p in zip(root.tolist(), depth.tolist(), path.tolist()):
        out.append(roots[r] + (format(p & ((1 << d) - 1), '0%db' % d) if d else ''))
    return out


def params_ref(p: native.VkCellParams):
    return ctypes.byref(p)
