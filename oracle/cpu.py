"""ctypes wrapper of oracle/liblens_oracle.so (TEST INFRASTRUCTURE / CPU BASELINE ONLY).

Numpy arrays in the same SoA layout as the device library; the table is the
compiled RateLawTable passed as a vk_table_desc of host pointers.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, 'liblens_oracle.so')

_i32p = ctypes.POINTER(ctypes.c_int32)
_f64p = ctypes.POINTER(ctypes.c_double)


class _Desc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        'n_species', 'n_dyn', 'n_reactions', 'n_rate_laws', 'n_params', 'n_ext',
        'n_sets', 'n_members', 'n_upd', 'n_exch')] + [
        ('rl_reaction', _i32p), ('rl_enzyme', _i32p), ('rl_kcat', _i32p),
        ('rl_num_ptr', _i32p), ('rl_den_ptr', _i32p), ('set_ptr', _i32p),
        ('mem_species', _i32p), ('mem_param', _i32p), ('upd_ptr', _i32p),
        ('upd_rxn', _i32p), ('upd_coeff', _f64p), ('ex_ptr', _i32p),
        ('ex_rxn', _i32p), ('ex_coeff', _f64p)]


def build():
    subprocess.run(['make', '-s', '-C', HERE], check=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        _lib.oc_rate_fluxes.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp]
        _lib.oc_step_euler.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_double, vp, vp, vp,
                                       vp, vp]
        _lib.oc_step_dopri5.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_double, ctypes.c_int, vp, vp, vp, vp,
                                        vp, vp, vp, vp]
        _lib.oc_step_dopri5.restype = ctypes.c_int
        _lib.oc_diffuse.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int]
        _lib.oc_exchange.argtypes = [vp, vp, vp, ctypes.c_int64, ctypes.c_double]
    return _lib


class Desc:
    """Keeps the numpy arrays alive for the life of the descriptor."""

    def __init__(self, table):
        self.keep = {}
        d = _Desc()
        d.n_species, d.n_dyn, d.n_reactions = table.n_species, table.n_dyn, table.n_reactions
        d.n_rate_laws, d.n_params, d.n_ext = table.n_rate_laws, table.n_params, table.n_ext
        d.n_sets = len(table.set_ptr) - 1
        d.n_members = len(table.mem_species)
        d.n_upd, d.n_exch = len(table.upd_rxn), len(table.ex_rxn)
        for name, arr in table.arrays().items():
            a = np.ascontiguousarray(arr)
            self.keep[name] = a
            setattr(d, name, a.ctypes.data_as(_f64p if a.dtype == np.float64 else _i32p))
        self.d = d

    @property
    def ptr(self):
        return ctypes.addressof(self.d)


def _p(a):
    return 0 if a is None else a.ctypes.data


def rate_fluxes(desc, params, conc, n=None):
    n = conc.shape[1] if n is None else n
    flux = np.zeros((desc.d.n_reactions, conc.shape[1]))
    lib().oc_rate_fluxes(desc.ptr, n, conc.shape[1], _p(params), _p(conc), _p(flux))
    return flux


def step_euler(desc, dt, params, conc, m2c, n=None):
    n = conc.shape[1] if n is None else n
    ld = conc.shape[1]
    flux = np.zeros((desc.d.n_reactions, ld))
    counts = np.zeros((desc.d.n_ext, ld), dtype=np.int64)
    lib().oc_step_euler(desc.ptr, n, ld, float(dt), _p(params), _p(conc), _p(m2c), _p(flux), _p(counts))
    return flux, counts


def step_dopri5(desc, dt, params, conc, m2c, h_state=None, rtol=1e-8, atol=1e-12, max_steps=100000,
                n=None):
    n = conc.shape[1] if n is None else n
    ld = conc.shape[1]
    flux = np.zeros((desc.d.n_reactions, ld))
    counts = np.zeros((desc.d.n_ext, ld), dtype=np.int64)
    status = np.zeros(ld, dtype=np.int32)
    nsteps = np.zeros(ld, dtype=np.int32)
    lib().oc_step_dopri5(desc.ptr, n, ld, float(dt), float(rtol), float(atol), int(max_steps),
                         _p(params), _p(conc), _p(m2c), _p(h_state), _p(flux), _p(counts),
                         _p(status), _p(nsteps))
    return flux, counts, status, nsteps


def diffuse(field, coef_dt, n_sub):
    """In place on a C-contiguous [nx, ny] float64 plane."""
    nx, ny = field.shape
    w0 = np.empty_like(field)
    w1 = np.empty_like(field)
    lib().oc_diffuse(_p(field), _p(w0), _p(w1), nx, ny, float(coef_dt), int(n_sub))
    return field


def exchange(field, bin_lin, counts, binvol_avogadro):
    lib().oc_exchange(_p(field), _p(np.ascontiguousarray(bin_lin, dtype=np.int32)),
                      _p(np.ascontiguousarray(counts, dtype=np.int64)), len(counts),
                      float(binvol_avogadro))
    return field
