#!/bin/bash
# Stage-split pass (variant 40): chunk rows that fill whole rounds of resident
# workgroups (5 per CU at 65 VGPRs: 1,280 on 256 CUs).  Whole C4 plane (76 tile
# columns x planes: 16 chunks per round) and one middle rank's band at N = 8 / 4 / 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-splitrounds}
mkdir -p $O
for w in 8 4 2; do
  case $w in
    8) SPEC=100:45:40:10,100:48:40:10,100:23:40:10; WV="20:34,40:256,40:128,40:86,40:64,40:52" ;;
    4) SPEC=100:77:40:10,100:39:40:10,100:96:40:10; WV="" ;;
    2) SPEC=100:135:40:10,100:68:40:10,100:64:40:10; WV="" ;;
  esac
  WHOLE_VARIANTS=$WV timeout -k 10 280 python scripts/rank_emulate.py $w --sweep $SPEC > $O/rank$w.log 2>&1 \
    || { tail -5 $O/rank$w.log; exit 2; }
  grep -v amdgpu.ids $O/rank$w.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print({k: d[k] for k in d if k in ('world','variant','rows','whole_plane_ms','graph_ms_per_step','graph_efficiency')})"
done
echo sweep-done
