#!/bin/bash
# A/B of the pair-sum pass's dispatch order (VK_STENCIL_EDGE_FIRST=0 / 1): the C4
# bench on one GPU, arms interleaved over rounds; then the order-1 stencil tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-orderab}
mkdir -p $O
for r in 1 2 3; do
  for o in 0 1; do
    VK_STENCIL_EDGE_FIRST=$o timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/c4_o${o}_$r.json 2> $O/c4_o${o}_$r.err \
      || { echo "arm $o failed"; tail -5 $O/c4_o${o}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/c4_o${o}_$r.json').read().strip().splitlines()[-1]); print('order $o round $r: %.4f ms/step, pass %s' % (d['ms_per_step'], d.get('roofline', {}).get('achieved')))"
  done
done
VK_STENCIL_EDGE_FIRST=1 timeout -k 10 500 python -u -m pytest tests/test_stencil_modes.py tests/test_configs.py tests/test_coupled_gpu.py tests/test_stencil_split.py -k "fma or c4_bench or coupled or bands" -x -q --timeout 300 --timeout-method thread > $O/pytest_o1.log 2>&1 || { tail -20 $O/pytest_o1.log; exit 2; }
tail -1 $O/pytest_o1.log
