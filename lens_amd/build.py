"""In-tree build of the HIP library (gfx950) -- no JIT cache, the .so travels with the repo.

    python -m lens_amd.build [--force]
"""

from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = sorted(glob.glob(os.path.join(HERE, 'csrc', '*.hip')))
HDRS = sorted(glob.glob(os.path.join(HERE, 'csrc', '*.h'))) + [os.path.join(REPO, 'include', 'vk_kinetics.h')]
OUT = os.path.join(HERE, 'lib', 'libvk_kinetics.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'

FLAGS = [
    '--offload-arch=' + ARCH, '-O3', '-std=c++17', '-fPIC', '-shared',
    # the exact kernels reproduce the reference's rounding sequence; FMAs are
    # written explicitly where a kernel wants them
    '-ffp-contract=off',
    '-Wall', '-Wno-unused-function',
    '-I' + os.path.join(REPO, 'include'), '-I' + os.path.join(HERE, 'csrc'),
    '-Wl,-rpath,/opt/rocm/lib', '-lhiprtc',
]


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if force or _stale(OUT, SRC + HDRS + [__file__]):
        cmd = [HIPCC] + FLAGS + SRC + ['-o', OUT + '.tmp']
        if verbose:
            print('[lens_amd.build]', ' '.join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    build(force='--force' in sys.argv)
