#!/bin/bash
# Default depth 10 in both modes: the full GPU record, then the exact-mode C4 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r04ag bash scripts/gpu_full.sh || exit 1
timeout -k 10 300 python -u bench.py --stencil-mode exact > gpurun_out/r04ag/bench_c4_exact.log 2>&1 || exit 2
tail -1 gpurun_out/r04ag/bench_c4_exact.log | cut -c1-200
