# GPU: SQ counters of the C4 kernels (K4s sort kernel) in separate --pmc passes, then
# C4 for the diagnostic builds in lib/variants/ under a kernel trace.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/pmcs && mkdir -p $O && rm -rf $O/*
run() { timeout -k 10 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  run 300 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 scripts/cbench.py --configs c4 --iters 1 --no-check --cpu-sample-c4 0 > $O/p$i.log 2>&1
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE
GROUPS
python3 scripts/pmc_summary.py $O/p1 $O/p2 | grep -A20 "canon_sort\|canon_table" | head -60
SKIP_TESTS=1 CONFIGS=c4 bash scripts/gpu_c4_trace.sh > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 1; }
for d in gpurun_out/c4t/default gpurun_out/c4t/libkmc_*; do [ -d $d ] || continue; echo "== $d"; python3 scripts/c4_calls.py $d | tail -1; done
