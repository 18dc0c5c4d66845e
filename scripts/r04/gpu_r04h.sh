#!/bin/bash
# r04h: coupled-pass A/B (gather placement, cached final pass) with tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_coupled_gpu.py > $O/pytest_coupled.log 2>&1 || { tail -40 $O/pytest_coupled.log; exit 6; }
tail -2 $O/pytest_coupled.log
timeout -k 10 300 python -u scripts/couple_ab.py 6 > $O/couple_ab.log 2>&1 || { tail -20 $O/couple_ab.log; exit 5; }
cat $O/couple_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/couple_ab.py 2 > $O/couple_ab_rocprof.log 2>&1 || { tail -20 $O/couple_ab_rocprof.log; exit 4; }
echo done
