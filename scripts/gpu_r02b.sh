# GPU (round 2, second call): full parity suite + smoke, C3/C4 with their parity
# checks under a kernel trace, PMC passes on the k = 13 radix pipeline (current R3).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r02b && rm -rf gpurun_out/r02b/*
O=gpurun_out/r02b
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cb -o cb -- python3 scripts/cbench.py --iters 3 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
grep '^{' $O/cb.log
run() { timeout -k 10 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  run 300 rocprofv3 --pmc $grp --output-format csv -d $O/pmc/p$i -o run -- python3 scripts/kbench.py --ks 13 --iters 2 > $O/pmc_p$i.log 2>&1
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
GROUPS
python3 scripts/pmc_summary.py $O/pmc > $O/pmc_summary.txt
cat $O/pmc_summary.txt
