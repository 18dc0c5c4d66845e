#!/bin/bash
# Stage-split pass (variant 40) chunk rows below 32: C3 on one GPU, whole C4 plane,
# and one middle rank's band at N = 8 / 4 / 2 (scripts/rank_emulate.py, no transfer).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-splitrows}
mkdir -p $O
SUB=c3 ROWS="${C3ROWS:-8 12 16 20}" timeout -k 10 280 bash scripts/c3_rows.sh > $O/c3_rows.log 2>&1 || { tail -5 $O/c3_rows.log; exit 1; }
cat $O/c3_rows.log
for w in 8 4 2; do
  WHOLE_VARIANTS=$([ $w = 8 ] && echo "20:34,40:16,40:24,40:32,40:64") timeout -k 10 280 python scripts/rank_emulate.py $w --sweep \
    100:16:40:10,100:24:40:10,100:32:40:10,100:48:40:10 > $O/rank$w.log 2>&1 || { tail -5 $O/rank$w.log; exit 2; }
  cat $O/rank$w.log
done
echo sweep-done
