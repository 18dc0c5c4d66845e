#!/bin/bash
# Full GPU session: every GPU test, smoke, the driver's bench command, and a rocprofv3
# kernel trace of the same command.  TAG names the output directory.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-full}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 3; }
tail -1 $O/bench_c4.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_c4_rocprof.log 2>&1 || { tail -20 $O/bench_c4_rocprof.log; exit 4; }
echo full-done
