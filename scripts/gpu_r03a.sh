# GPU (round 3, first pass): parity suite, the bench line at N = 1 and the N = 2
# rehearsal with its new fields, the concurrent-kernel experiment, fresh LDS
# counters of the k = 8 kernel, per-shard HBM traffic, config C1, per-rank steps.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03a && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit 1; }
tail -1 $O/gpu_tests.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 600 python bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-300
KMC_BENCH_BACKEND=gloo run 600 python bench.py --gpus 2 --steps 5 --warmup 3 --cpu-sample 2000000 > $O/bench_gloo2.log 2>&1
grep "^{" $O/bench_gloo2.log | cut -c1-200
run 300 python scripts/interfere.py > $O/interfere.log 2>&1
grep "^{" $O/interfere.log
run 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_lds -o run -- python3 scripts/kbench.py --ks 8 --iters 3 > $O/pmc_lds.log 2>&1
run 200 rocprofv3 --pmc SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_lds2 -o run -- python3 scripts/kbench.py --ks 8 --iters 3 > $O/pmc_lds2.log 2>&1
python3 scripts/pmc_summary.py $O/pmc_lds $O/pmc_lds2 > $O/pmc_lds_summary.txt
grep -A20 "count_dense_kernel<8, 1, 3" $O/pmc_lds_summary.txt
run 300 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_128B --output-format csv -d $O/pmc_fetch -o run -- python3 scripts/pmc_shards.py run > $O/pmc_shards_run.log 2>&1
run 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 scripts/pmc_shards.py run > $O/pmc_shards_run2.log 2>&1
python3 scripts/pmc_shards.py parse $O/pmc_fetch $O/pmc_write $O/pmc_shards_run.log $O/pmc_dense_k8_shards.json
run 300 python scripts/cbench.py --configs c1 > $O/c1.log 2>&1
grep "^{" $O/c1.log | cut -c1-400
run 300 python scripts/shardbench.py --worlds 1,1,2,4,8 > $O/shard.log 2>&1
grep '^{' $O/shard.log | cut -c1-200
