# GPU: PMC passes over the k = 13 radix pipeline (scripts/kbench.py --ks 13).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${PMC_OUT:-pmc_c3} && mkdir -p $O && rm -rf $O/*
run() { timeout -k 10 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  run 300 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 scripts/kbench.py --ks ${KS:-13} --iters 2 > $O/p$i.log 2>&1
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES
GROUPS
python3 scripts/pmc_summary.py $O > $O/summary.txt
cat $O/summary.txt
