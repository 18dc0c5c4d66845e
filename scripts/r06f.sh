set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum SQ_WAVES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_BUSY_CYCLES GRBM_GUI_ACTIVE; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o run -- python3 scripts/c4_kin_once.py > $O/pmc_$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 $O/pmc_$i.log; exit 6; }
done
echo pmc-done
