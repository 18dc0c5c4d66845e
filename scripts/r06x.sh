#!/bin/bash
# Round-6 session x: the image-based exchange in the final pass -- its GPU tests, an
# exin / separate-sweep A/B, and the rocprof per-step kernel sums of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06x}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_exchange_in_pass.py tests/test_coupled_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=$T ROUNDS=${ROUNDS:-4} ARMS="exin:--steps 30|sep:--no-exchange-in-pass --steps 30" bash scripts/bench_arms.sh || exit 2
TAG=$T ARMS="exin:|sep:--no-exchange-in-pass" bash scripts/prof_arms.sh || exit 3
echo session-done
