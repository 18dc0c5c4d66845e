set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stencil_modes.py tests/test_gpu_parity.py tests/test_stencil_split.py tests/test_coupled_gpu.py tests/test_bench_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_stencil.log 2>&1 || { tail -30 $O/pytest_stencil.log; exit 1; }
tail -2 $O/pytest_stencil.log
timeout -k 10 400 python bench.py > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 3; }
tail -1 $O/bench_c4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('copy_floor')); print(json.dumps(d.get('secondary'), indent=1))"
