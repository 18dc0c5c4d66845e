"""In-tree build of the HIP library (gfx950) -- no JIT cache, the .so travels with the repo.

    python -m lens_amd.build [--force]
"""

from __future__ import annotations

import glob
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = sorted(glob.glob(os.path.join(HERE, 'csrc', '*.hip')))
HDRS = sorted(glob.glob(os.path.join(HERE, 'csrc', '*.h')) + glob.glob(os.path.join(HERE, 'csrc', '*.inc'))) + [os.path.join(REPO, 'include', 'vk_kinetics.h')]
OUT = os.path.join(HERE, 'lib', 'libvk_kinetics.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'

COMPILE = [
    '--offload-arch=' + ARCH, '-O3', '-std=c++17', '-fPIC',
    # the exact kernels reproduce the reference's rounding sequence; FMAs are
    # written explicitly where a kernel wants them
    '-ffp-contract=off',
    '-Wall', '-Wno-unused-function',
    '-I' + os.path.join(REPO, 'include'), '-I' + os.path.join(HERE, 'csrc'),
]
# Per-unit extra flags.  The pair-sum passes keep v_fma_f64 (three-address) instead of
# v_fmac_f64 (same bits): the accumulator-tied fmac forced 30 register copies per 6 rows
# of the 10-deep steady loop (642 -> 612 VALU instructions, same VGPRs; C4 1.255-1.263
# -> 1.240-1.250 ms per step, profiles/r06/nofmac).  Kremling sheds 458 copies the same
# way but runs no faster (r06/kremab), so it keeps the default
EXTRA = {name: ['-Xclang', '-target-feature', '-Xclang', '-fmacf64-inst']
         for name in ('vk_stencil_ps.hip', 'vk_stencil_ps10.hip', 'vk_stencil_sp.hip')}
LINK = ['--offload-arch=' + ARCH, '-shared', '-fPIC', '-Wl,--no-undefined', '-Wl,-rpath,/opt/rocm/lib', '-lhiprtc']
OBJ_DIR = os.path.join(HERE, 'lib', 'obj')


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if force or _stale(OUT, SRC + HDRS + [__file__]):
        # one hipcc per translation unit, in parallel (the stencil launchers are
        # split over several units so their template instantiations spread out)
        os.makedirs(OBJ_DIR, exist_ok=True)
        objs = [os.path.join(OBJ_DIR, os.path.basename(src)[:-4] + '.o') for src in SRC]
        todo = [(src, obj) for src, obj in zip(SRC, objs) if force or _stale(obj, [src] + HDRS + [__file__])]
        jobs = max(1, min(len(todo), int(os.environ.get('MAX_JOBS', '0')) or (os.cpu_count() or 1)))

        def compile_one(pair):
            cmd = [HIPCC] + COMPILE + EXTRA.get(os.path.basename(pair[0]), []) + ['-c', pair[0], '-o', pair[1] + '.tmp']
            if verbose:
                print('[lens_amd.build]', ' '.join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            os.replace(pair[1] + '.tmp', pair[1])

        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(compile_one, todo))
        cmd = [HIPCC] + LINK + objs + ['-o', OUT + '.tmp']
        if verbose:
            print('[lens_amd.build]', ' '.join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    build(force='--force' in sys.argv)
