"""The C-ABI library loads and exports every symbol include/vk_kinetics.h declares
(no compute calls: this runs without a GPU)."""

import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, 'include', 'vk_kinetics.h')


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:int|int64_t|const char \*)\s*(vk_\w+)\s*\(', text, re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    assert 'vk_step_dopri5' in syms and 'vk_diffuse' in syms and len(syms) >= 13


def test_library_exports_every_declared_symbol():
    from lens_amd import native
    from lens_amd.build import build
    build(verbose=False)
    lib = ctypes.CDLL(native.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert set(declared_symbols()) == set(native.EXPORTS)
    lib.vk_abi_version.restype = ctypes.c_int
    assert lib.vk_abi_version() == 1


def test_library_is_gfx950_code_object():
    from lens_amd import native
    data = open(native.LIB_PATH, 'rb').read()
    assert b'gfx950' in data


def test_product_never_imports_the_oracle():
    pkg = os.path.join(REPO, 'lens_amd')
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(('.py', '.hip', '.h', '.cpp')):
                src = open(os.path.join(root, f)).read()
                assert 'oracle' not in re.sub(r'#.*|//.*|""".*?"""', '', src, flags=re.S), f


def test_missing_library_fails_loudly(tmp_path):
    from lens_amd import native
    with pytest.raises(native.NativeError):
        native.load.__wrapped__(str(tmp_path / 'nope.so')) if hasattr(native.load, '__wrapped__') \
            else _load_fresh(native, str(tmp_path / 'nope.so'))


def _load_fresh(native, path):
    saved = native._lib
    native._lib = None
    try:
        native.load(path)
    finally:
        native._lib = saved


def test_bench_uses_the_oracle_only_in_its_cpu_baseline():
    """bench.py may import oracle/ only inside its CPU-baseline functions (after the
    timed GPU region), never to build or run the measured workload."""
    import ast
    tree = ast.parse(open(os.path.join(REPO, 'bench.py')).read())
    for fn in ast.walk(tree):
        if isinstance(fn, ast.FunctionDef):
            for node in ast.walk(fn):
                if isinstance(node, (ast.Import, ast.ImportFrom)):
                    names = [a.name for a in node.names] + [getattr(node, 'module', None) or '']
                    if any(n.split('.')[0] == 'oracle' for n in names):
                        assert fn.name.startswith('cpu_baseline'), fn.name
    top = [n for n in tree.body if isinstance(n, (ast.Import, ast.ImportFrom))]
    assert not any('oracle' in (getattr(n, 'module', '') or '') or any('oracle' in a.name for a in n.names)
                   for n in top)
