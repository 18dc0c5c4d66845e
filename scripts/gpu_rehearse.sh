set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_distributed_gpu.py > gpurun_out/dist_gpu.log 2>&1 || { tail -30 gpurun_out/dist_gpu.log; exit 3; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline > gpurun_out/rehearsal_c4_2r.log 2>&1 || { tail -30 gpurun_out/rehearsal_c4_2r.log; exit 4; }
echo ok
