#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group; kernel-trace only, no sys/runtime trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD=${CMD:-python3 scripts/stencil_once.py}
TAG=${TAG:-pmc}
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_$i -o run -- $CMD > gpurun_out/${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/${TAG}_$i.log; exit 6; }
done
echo pmc-done
