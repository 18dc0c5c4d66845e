#!/bin/bash
# Edge-first tile order in every pass kernel: the stencil / band / coupled / config
# GPU tests, the C4 and C3 benches, one middle rank per N, and a rows sweep of the
# whole C4 plane.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05w}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stencil_modes.py tests/test_stencil_split.py tests/test_coupled_gpu.py tests/test_configs.py tests/test_distributed_gpu.py tests/test_graph_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in c4 c3; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 20 > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 2; }
  python -c "import json; d=json.loads(open('$O/$w.json').read().strip().splitlines()[-1]); print('$w %.4f ms/step %.3e  pass %s GB/s frac %s' % (d['ms_per_step'], d['value'], d['roofline']['achieved'], d['roofline']['frac']))"
done
for w in 8 4 2; do
  WHOLE_VARIANTS=$([ $w = 8 ] && echo "20:34,20:40,20:48,20:64,20:86,40:52,40:64,40:86") timeout -k 10 280 python scripts/rank_emulate.py $w --sweep 100:0:40:10,100:0:20:10 > $O/rank$w.log 2>&1 || { tail -5 $O/rank$w.log; exit 3; }
  grep -v amdgpu.ids $O/rank$w.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print({k: d[k] for k in d if k in ('world','variant','rows','whole_plane_ms','graph_ms_per_step','graph_efficiency')})"
done
echo w-done
