# GPU: SQ/LDS PMC groups over the C4 canonical kernels (one counter group per rocprofv3 run).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc4 && rm -rf gpurun_out/pmc4/*
run() { timeout -k 10 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  KMC_LIB=${KMC_LIB:-} run 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc4/p$i -o run -- python3 scripts/cbench.py --configs ${CONFIGS:-c4} --iters 1 --cpu-sample-c4 0 --cpu-sample-c3 0 > gpurun_out/pmc4/p$i.log 2>&1
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM
FETCH_SIZE
WRITE_SIZE
GROUPS
python3 scripts/pmc_summary.py gpurun_out/pmc4 > gpurun_out/pmc4/summary.txt
grep -A26 "canon_\|radix_" gpurun_out/pmc4/summary.txt | head -150
