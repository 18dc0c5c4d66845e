#!/bin/bash
# rocprofv3 kernel trace of bench.py per argument set (ARMS as bench_arms.sh), and the
# per-step kernel sums (scripts/step_kernel_sum.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-profarms}; mkdir -p $O
export TMPDIR=/tmp
IFS='|' read -ra A <<< "$ARMS"
for arm in "${A[@]}"; do
  lab=${arm%%:*}; args=${arm#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lab -o run -- \
    python3 bench.py --no-cpu-baseline --secondary-steps 0 --steps 20 $args > $O/bench_$lab.log 2>&1 || { echo "prof $lab failed"; tail -5 $O/bench_$lab.log; exit 1; }
  python3 scripts/step_kernel_sum.py $O/prof_$lab/run_kernel_trace.csv > $O/steps_$lab.json || exit 2
  echo "== $lab"; tail -1 $O/bench_$lab.log | cut -c1-120; python3 -c "import json; d=json.load(open('$O/steps_$lab.json')); print(d['median_step_kernel_ms'], d['median_step_span_ms'], d['per_kernel_median_ms_per_step'])"
done
echo prof-done
