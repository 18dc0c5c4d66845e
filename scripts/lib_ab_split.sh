#!/bin/bash
# A/B of two library builds (lens_amd/lib/ab_base.so, ab_new.so) on the split-pass
# workloads: the C3 bench and one middle rank's band at N = 8 / 4 (graph-replayed,
# scripts/rank_emulate.py), interleaved rounds; the new build is left installed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-libabsplit}; mkdir -p $O
for r in 1 2; do
  for arm in ${ARMS:-base new}; do
    cp lens_amd/lib/ab_$arm.so lens_amd/lib/libvk_kinetics.so
    timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline --steps 40 > $O/c3_${arm}_$r.json 2> $O/c3_${arm}_$r.err \
      || { echo "arm $arm failed"; tail -5 $O/c3_${arm}_$r.err; exit 1; }
    c3=$(python -c "import json; d=json.loads(open('$O/c3_${arm}_$r.json').read().strip().splitlines()[-1]); print('%.4f' % d['ms_per_step'])")
    for w in 8 4; do
      timeout -k 10 200 python scripts/rank_emulate.py $w --sweep 100:0:40:10 > $O/rank${w}_${arm}_$r.log 2>&1 || { tail -5 $O/rank${w}_${arm}_$r.log; exit 2; }
    done
    b8=$(grep graph_ms $O/rank8_${arm}_$r.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['graph_ms_per_step'])")
    b4=$(grep graph_ms $O/rank4_${arm}_$r.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['graph_ms_per_step'])")
    echo "$arm round $r: C3 $c3 ms/step, N=8 band $b8 ms, N=4 band $b4 ms"
  done
done
