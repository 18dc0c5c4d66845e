set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 120 ./scripts/micro/mall_bw > $O/mall_bw.log 2>&1 || { tail $O/mall_bw.log; exit 1; }
cat $O/mall_bw.log
for n in 4096 2896 2048 1448; do
  timeout -k 10 200 python scripts/stencil_sweep.py $n 20:10:64:1,20:10:32:1,20:10:16:1,40:10:0:1 > $O/sweep_$n.log 2>&1 || { tail $O/sweep_$n.log; exit 2; }
  echo "n=$n"; grep variant $O/sweep_$n.log
done
