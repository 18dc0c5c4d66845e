#!/bin/bash
# Round-6 session h: the lookahead-skip pass (no loads past a chunk's cone):
# stencil GPU tests on the new build, base/new A/B on the C4 bench, FETCH_SIZE of the new pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06h}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cp lens_amd/lib/ab_new.so lens_amd/lib/libvk_kinetics.so
TAG=$T/st bash scripts/gpu_stencil_tests.sh || exit 1
TAG=$T/ab ARMS="base new" bash scripts/lib_ab.sh || exit 2
for arm in base new; do
  cp lens_amd/lib/ab_$arm.so lens_amd/lib/libvk_kinetics.so
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$arm -o run -- \
    python3 scripts/stencil_once.py > $O/pmc_fetch_$arm.log 2>&1 || { echo "pmc $arm failed"; tail -5 $O/pmc_fetch_$arm.log; exit 3; }
done
echo session-done
