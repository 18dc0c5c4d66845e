set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_stencil_split.py tests/test_configs.py -k "split or c3_bench or bands" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 150 python bench.py --workload c3 --no-cpu-baseline --steps 40 --warmup 5 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 2; }
tail -1 $O/c3.json | cut -c1-300
timeout -k 10 280 python scripts/rank_emulate.py 8 --sweep 100:0:40:10 > $O/rank8.log 2>&1 || exit 3
timeout -k 10 280 python scripts/rank_emulate.py 4 --sweep 100:0:40:10 > $O/rank4.log 2>&1 || exit 3
timeout -k 10 280 python scripts/rank_emulate.py 2 --sweep 100:0:40:10 > $O/rank2.log 2>&1 || exit 3
grep -h graph_ms $O/rank*.log | cut -c1-260
