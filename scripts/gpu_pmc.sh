# GPU: PMC counter passes over the dense kernels (one counter group per rocprofv3 run).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc && rm -rf gpurun_out/pmc/*
run() { timeout -k 10 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
LIB=${LIB:-$PWD/dna-kmeres-parallel_amd/lib/libkmc.so}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  KMC_LIB=$LIB run 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 scripts/kbench.py --ks ${KS:-3,7,8} --iters 2 > gpurun_out/pmc/p$i.log 2>&1
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN
FETCH_SIZE
WRITE_SIZE
GROUPS
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt
grep -A40 "count_dense_kernel" gpurun_out/pmc/summary.txt | head -150
