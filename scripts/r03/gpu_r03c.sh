#!/bin/bash
# Round-3 session c: graph-timing test, multi-rank graph tests, C4 bench (fma
# default + exact), a rocprofv3 kernel-trace of the driver's own command, PMC
# passes of the fma pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03c
export VK_FLIPS_LOG=$PWD/gpurun_out/${T}_flips.jsonl
rm -f $VK_FLIPS_LOG
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_engine_gpu.py tests/test_registry.py tests/test_distributed_gpu.py tests/test_configs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${T}_c4.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4.log; exit 2; }
tail -1 gpurun_out/bench_${T}_c4.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --stencil-mode exact --no-cpu-baseline > gpurun_out/bench_${T}_c4_exact.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4_exact.log; exit 3; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T} -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${T}.log 2>&1 || { tail -20 gpurun_out/prof_${T}.log; exit 4; }
export VARIANT=6 DEPTH=9 ROWS=64 REPS=2 MODE=fma
i=0
for grp in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,GRBM_GUI_ACTIVE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- python3 scripts/stencil_once.py > gpurun_out/pmc_${T}_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 gpurun_out/pmc_${T}_$i.log; exit 6; }
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --workload c3 --dist-backend gloo > gpurun_out/${T}_rehearse_c3.log 2>&1 || { tail -20 gpurun_out/${T}_rehearse_c3.log; exit 7; }
tail -1 gpurun_out/${T}_rehearse_c3.log | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 20 --warmup 5 --workload c2 --dist-backend gloo > gpurun_out/${T}_rehearse_c2.log 2>&1 || { tail -20 gpurun_out/${T}_rehearse_c2.log; exit 8; }
tail -1 gpurun_out/${T}_rehearse_c2.log | cut -c1-300
echo session-done
