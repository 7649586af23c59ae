# GPU call: kernel micro-bench (normal + ablation builds), counter list, kernel trace, PMC passes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/prof
set -o pipefail
run() { timeout -k 10 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 300 python scripts/kbench.py --ks 1,2,3,4,5,6,7,8 > gpurun_out/kbench.log 2>&1
KMC_LIB=$PWD/dna-kmeres-parallel_amd/lib/libkmc_abl1.so run 200 python scripts/kbench.py --ks 3,7,8 >> gpurun_out/kbench.log 2>&1
KMC_LIB=$PWD/dna-kmeres-parallel_amd/lib/libkmc_abl2.so run 200 python scripts/kbench.py --ks 3,7,8 >> gpurun_out/kbench.log 2>&1
grep -v amdgpu.ids gpurun_out/kbench.log
run 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
run 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o k8 -- python3 scripts/kbench.py --ks 8 --iters 5 > gpurun_out/prof_trace.log 2>&1
run 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/prof/pmc1 -o k8 -- python3 scripts/kbench.py --ks 8 --iters 2 > gpurun_out/prof_pmc1.log 2>&1
run 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/pmc2 -o k8 -- python3 scripts/kbench.py --ks 8 --iters 2 > gpurun_out/prof_pmc2.log 2>&1
run 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc3 -o k8 -- python3 scripts/kbench.py --ks 8 --iters 2 > gpurun_out/prof_pmc3.log 2>&1
run 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc4 -o k8 -- python3 scripts/kbench.py --ks 8 --iters 2 > gpurun_out/prof_pmc4.log 2>&1
echo done
