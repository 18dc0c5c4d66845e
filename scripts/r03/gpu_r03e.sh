#!/bin/bash
# Round-3 session e: C5 branch-free publish A/B + bit-identity, C4 bench with the eager-step split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r03e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "wave_spec_equals" -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 600 python -u scripts/c5_probe.py > gpurun_out/${T}_c5_probe.log 2>&1 || { tail -20 gpurun_out/${T}_c5_probe.log; exit 2; }
cat gpurun_out/${T}_c5_probe.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${T}_c4.log 2>&1 || { tail -20 gpurun_out/bench_${T}_c4.log; exit 3; }
tail -1 gpurun_out/bench_${T}_c4.log | cut -c1-200
for n in 2 4 8; do
  timeout -k 10 120 python scripts/rank_emulate.py $n 100 0 6 9 fma >> gpurun_out/${T}_rank_emulate.log 2>&1 || { tail -5 gpurun_out/${T}_rank_emulate.log; exit 4; }
done
timeout -k 10 120 python scripts/rank_emulate.py 8 100 16 6 9 fma >> gpurun_out/${T}_rank_emulate.log 2>&1 || { tail -5 gpurun_out/${T}_rank_emulate.log; exit 4; }
timeout -k 10 120 python scripts/rank_emulate.py 8 100 32 6 9 fma >> gpurun_out/${T}_rank_emulate.log 2>&1 || { tail -5 gpurun_out/${T}_rank_emulate.log; exit 4; }
grep ms/step gpurun_out/${T}_rank_emulate.log
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/${T}_counters_avail.txt 2>&1 || true
grep -io "SQC_ICACHE[A-Z_]*" gpurun_out/${T}_counters_avail.txt | sort -u | head
echo session-done
# last: an instruction-cache counter pass on the 9-deep fma stencil pass (nothing runs after it)
export VARIANT=6 DEPTH=9 ROWS=64 REPS=2 MODE=fma
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_${T}_icache -o run -- python3 scripts/stencil_once.py > gpurun_out/pmc_${T}_icache.log 2>&1
echo icache-pass rc=$?
