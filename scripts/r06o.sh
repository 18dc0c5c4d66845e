#!/bin/bash
# Round-6 session o: the exchange added in the final pass (vk_diffuse_exchange): its
# parity tests and the neighbouring suites, then an on/off A/B on the C4 bench and the
# rocprof per-step kernel sums of both arms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06o}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_exchange_in_pass.py tests/test_coupled_gpu.py tests/test_stencil_modes.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=$T ROUNDS=3 ARMS="exin:--steps 30|sep:--no-exchange-in-pass --steps 30" bash scripts/bench_arms.sh || exit 2
TAG=$T ARMS="exin:|sep:--no-exchange-in-pass" bash scripts/prof_arms.sh || exit 3
echo session-done
