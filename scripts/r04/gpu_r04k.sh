#!/bin/bash
# r04k: overlapped capture -- graph / coupled / C4 bench-configuration tests, the A/B, the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py tests/test_coupled_gpu.py "tests/test_configs.py::test_c4_bench_configuration_full_step_vs_c_oracle" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 6; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/couple_ab.py 6 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 5; }
cat $O/ab.log
timeout -k 10 400 python bench.py > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 3; }
tail -1 $O/bench_c4.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_c4_rocprof.log 2>&1 || { tail -20 $O/bench_c4_rocprof.log; exit 4; }
echo done
