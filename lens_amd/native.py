"""ctypes binding of the C ABI in ``include/vk_kinetics.h``.

The shared library ``lens_amd/lib/libvk_kinetics.so`` is built in-tree by
``lens_amd/build.py`` (hipcc, gfx950).  There is no fallback: if the library
is missing or a call fails, a :class:`NativeError` is raised.

torch is imported before the library is loaded so that the HIP runtime torch
ships (SONAME ``libamdhip64.so.7``) is the one the library binds to -- device
pointers from torch tensors and torch's stream handles are then valid for
every vk_* call.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib')
LIB_PATH = os.environ.get('VK_KINETICS_LIB') or os.path.join(LIB_DIR, 'libvk_kinetics.so')   # env: A/B builds

VK_OK, VK_ERR_ARG, VK_ERR_HIP, VK_ERR_LIMIT, VK_ERR_NOMEM = 0, 1, 2, 3, 4
VK_AGENT_MAX_STEPS, VK_AGENT_H_UNDERFLOW, VK_AGENT_NONFINITE = 1, 2, 4

# every symbol include/vk_kinetics.h declares (tests check the exports)
EXPORTS = (
    'vk_abi_version', 'vk_last_error', 'vk_table_create', 'vk_table_destroy', 'vk_table_specialize',
    'vk_rate_fluxes', 'vk_step_euler', 'vk_step_dopri5', 'vk_step_dopri5_multi', 'vk_step_dopri5_gather', 'vk_field_uniform',
    'vk_diffuse', 'vk_diffuse_part', 'vk_diffuse_delta', 'vk_diffuse_coupled', 'vk_set_stencil_depth', 'vk_set_stencil_kernel', 'vk_set_stencil_mode',
    'vk_timestamp', 'vk_wall_clock_khz', 'vk_copy_stream', 'vk_gather', 'vk_exchange_sorted',
    'vk_exchange_atomic', 'vk_bin_sites', 'vk_cell_step', 'vk_divide_scratch_bytes', 'vk_divide_plan',
    'vk_divide_gather', 'vk_divide_lineage', 'vk_divide_locations', 'vk_kremling_step',
    'vk_expression_step',
)

VK_CELL_MASS, VK_CELL_VOLUME, VK_CELL_LENGTH, VK_CELL_SURFACE_AREA, VK_CELL_PROTEIN, VK_CELL_ANGLE = range(6)
VK_CELL_ROWS = 6
VK_GROWTH_PROTEIN, VK_GROWTH_MASS = 0, 1
VK_RNG_STREAM, VK_RNG_PHILOX = 0, 1
VK_DIVIDE_SET, VK_DIVIDE_SPLIT, VK_DIVIDE_ZERO = 0, 1, 2
VK_UNIFORM_BLOCKS = 512
VK_PART_ALL, VK_PART_INTERIOR, VK_PART_EDGES = 0, 1, 2


class NativeError(RuntimeError):
    pass


_i32p = ctypes.POINTER(ctypes.c_int32)
_f64p = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f64 = ctypes.c_double


class VkTableDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        'n_species', 'n_dyn', 'n_reactions', 'n_rate_laws', 'n_params', 'n_ext',
        'n_sets', 'n_members', 'n_upd', 'n_exch')] + [
        ('rl_reaction', _i32p), ('rl_enzyme', _i32p), ('rl_kcat', _i32p),
        ('rl_num_ptr', _i32p), ('rl_den_ptr', _i32p), ('set_ptr', _i32p),
        ('mem_species', _i32p), ('mem_param', _i32p), ('upd_ptr', _i32p),
        ('upd_rxn', _i32p), ('upd_coeff', _f64p), ('ex_ptr', _i32p),
        ('ex_rxn', _i32p), ('ex_coeff', _f64p)]


class VkOdeOpts(ctypes.Structure):
    _fields_ = [('rtol', ctypes.c_double), ('atol', ctypes.c_double),
                ('max_steps', ctypes.c_int32), ('variant', ctypes.c_int32)]


class VkCellParams(ctypes.Structure):
    _fields_ = [('model', ctypes.c_int32), ('rng', ctypes.c_int32)] + [
        (n, ctypes.c_double) for n in (
            'factor', 'divide_protein', 'division_volume', 'protein_mw', 'avogadro', 'fg_per_g',
            'density', 'volume_to_fl', 'cap_volume', 'cap_area', 'two_r', 'width', 'sa_const',
            'sa_lin')] + [('seed', ctypes.c_uint64), ('step', ctypes.c_uint64)]


class VkKremlingParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        'k1', 'k2', 'k3', 'K1', 'K2', 'K3', 'kd', 'm', 'n', 'x0', 'kg6p', 'Kg6p', 'kptsup', 'Kglc',
        'Keiiap', 'klac', 'Km_lac', 'Kieiia', 'kgly', 'kpyk', 'kpdh', 'kpts', 'km_pts', 'mw1', 'mw2',
        'mw3', 'Y1_sim', 'Y2_sim', 'Y3_sim', 'K', 'kb', 'ksyn', 'KI')]


_SIGS = {
    'vk_abi_version': ([], ctypes.c_int),
    'vk_last_error': ([], ctypes.c_char_p),
    'vk_table_create': ([ctypes.POINTER(VkTableDesc), ctypes.POINTER(_vp)], ctypes.c_int),
    'vk_table_destroy': ([_vp], ctypes.c_int),
    'vk_table_specialize': ([_vp, ctypes.c_char_p], ctypes.c_int),
    'vk_rate_fluxes': ([_vp, _i64, _i64, _vp, _vp, _vp, _vp], ctypes.c_int),
    'vk_step_euler': ([_vp, _i64, _i64, _f64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], ctypes.c_int),
    'vk_step_dopri5': ([_vp, _i64, _i64, _f64, ctypes.POINTER(VkOdeOpts), _vp, _vp, _vp, _vp,
                        _vp, _vp, _vp, _vp, _vp, _vp], ctypes.c_int),
    'vk_step_dopri5_multi': ([_vp, _i64, _i64, _f64, _i32, ctypes.POINTER(VkOdeOpts), _vp, _vp, _vp, _vp, _vp,
                              _i64, _vp, _i64, _vp, _vp, _i64, _vp], ctypes.c_int),
    'vk_step_dopri5_gather': ([_vp, _i64, _i64, _f64, ctypes.POINTER(VkOdeOpts), _vp, _vp, _vp, _vp, _vp, _vp,
                               _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i32, _vp], ctypes.c_int),
    'vk_field_uniform': ([_vp, _i32, _i64, _i32, _i32, _i32, _vp, _vp, _vp], ctypes.c_int),
    'vk_diffuse': ([_vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                    _i32, _i32, _i32, _f64, _vp, _vp], ctypes.c_int),
    'vk_diffuse_part': ([_vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                         _i32, _i32, _i32, _f64, _vp, _i32, _i32, _vp], ctypes.c_int),
    'vk_diffuse_delta': ([_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                          _i32, _i32, _i32, _f64, _vp, _vp], ctypes.c_int),
    'vk_diffuse_coupled': ([_vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _f64, _vp, _vp, _vp, _i32, _i64,
                            _i32p, _vp, _i64, _i32p, _vp, _i64, _f64, _vp], ctypes.c_int),
    'vk_set_stencil_depth': ([_i32], ctypes.c_int),
    'vk_set_stencil_kernel': ([_i32, _i32], ctypes.c_int),
    'vk_set_stencil_mode': ([_i32], ctypes.c_int),
    'vk_timestamp': ([_vp, _i32, _vp], ctypes.c_int),
    'vk_wall_clock_khz': ([], ctypes.c_int64),
    'vk_copy_stream': ([_vp, _vp, _i64, _vp], ctypes.c_int),
    'vk_gather': ([_vp, _i64, _vp, _i64, _vp, _vp, _i32, _vp, _i64, _vp], ctypes.c_int),
    'vk_exchange_sorted': ([_vp, _i64, _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _i32, _f64, _vp],
                           ctypes.c_int),
    'vk_exchange_atomic': ([_vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _f64, _vp], ctypes.c_int),
    'vk_bin_sites': ([_vp, _i64, _i64, _i32, _i32, _f64, _f64, _i32, _vp, _vp, _vp], ctypes.c_int),
    'vk_cell_step': ([ctypes.POINTER(VkCellParams), _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
                     ctypes.c_int),
    'vk_divide_scratch_bytes': ([_i64], ctypes.c_int64),
    'vk_divide_plan': ([_vp, _i64, _vp, _vp, _vp, _vp, _vp], ctypes.c_int),
    'vk_divide_gather': ([_i64, _vp, _vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _vp], ctypes.c_int),
    'vk_divide_lineage': ([_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], ctypes.c_int),
    'vk_divide_locations': ([_i64, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp], ctypes.c_int),
    'vk_expression_step': ([_vp, _i64, _i64, _f64, _vp, _vp, _vp, _i32, _vp], ctypes.c_int),
    'vk_kremling_step': ([ctypes.POINTER(VkKremlingParams), _i64, _i64, _f64, _f64, _i32, _f64, _f64, _i32,
                          _vp, _vp, _f64, _vp, _vp, _vp, _vp, _vp, _vp], ctypes.c_int),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load (once) and return the library handle.  Raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeError(
            '%s is missing: build it with `python -c "import __graft_entry__ as g; g.build()"` '
            '(there is no CPU fallback)' % path)
    import torch  # noqa: F401  -- bind to torch's HIP runtime (see module doc)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.vk_abi_version() != 1:
        raise NativeError('ABI version mismatch')
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != VK_OK:
        msg = _lib.vk_last_error().decode(errors='replace') if _lib else ''
        raise NativeError('%s failed (status %d): %s' % (what, rc, msg))


def ptr(t) -> int:
    """Device pointer of a torch tensor (None -> NULL)."""
    return 0 if t is None else t.data_ptr()


def resolve_device(device=None):
    """torch.device with an explicit index: ``'cuda'`` -> ``cuda:<current>``.

    Tensors always report an indexed device, and ``cuda != cuda:0`` in torch,
    so every engine keeps the indexed form (Colony(device='cuda'))."""
    import torch
    if device is None:
        return torch.device('cuda', torch.cuda.current_device())
    d = torch.device(device)
    if d.type == 'cuda' and d.index is None:
        return torch.device('cuda', torch.cuda.current_device())
    return d


def stream_handle(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


class DeviceTable:
    """Owns a vk_table compiled from a :class:`RateLawTable`."""

    def __init__(self, table):
        lib = load()
        self.table = table
        self._keep = []

        def ip(a):
            a = np.ascontiguousarray(a, dtype=np.int32)
            self._keep.append(a)
            return a.ctypes.data_as(_i32p)

        def dp(a):
            a = np.ascontiguousarray(a, dtype=np.float64)
            self._keep.append(a)
            return a.ctypes.data_as(_f64p)

        d = VkTableDesc()
        d.n_species, d.n_dyn, d.n_reactions = table.n_species, table.n_dyn, table.n_reactions
        d.n_rate_laws, d.n_params, d.n_ext = table.n_rate_laws, table.n_params, table.n_ext
        d.n_sets = len(table.set_ptr) - 1
        d.n_members = len(table.mem_species)
        d.n_upd = len(table.upd_rxn)
        d.n_exch = len(table.ex_rxn)
        for name in ('rl_reaction', 'rl_enzyme', 'rl_kcat', 'rl_num_ptr', 'rl_den_ptr', 'set_ptr',
                     'mem_species', 'mem_param', 'upd_ptr', 'upd_rxn', 'ex_ptr', 'ex_rxn'):
            setattr(d, name, ip(getattr(table, name)))
        d.upd_coeff = dp(table.upd_coeff)
        d.ex_coeff = dp(table.ex_coeff)
        h = _vp()
        check(lib.vk_table_create(ctypes.byref(d), ctypes.byref(h)), 'vk_table_create')
        self.handle = h
        self._keep = []

    def close(self):
        if getattr(self, 'handle', None) and _lib is not None:
            _lib.vk_table_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
