# GPU: rocprofv3 kernel trace + HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes)
# of the bench command itself; summaries land in gpurun_out/prof_bench/ and are
# copied into profiles/ by scripts/profile_summary.py (run on the build host).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/prof_bench && rm -rf gpurun_out/prof_bench/*
run() { timeout -k 10 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
ARGS="--steps ${STEPS:-20} --warmup 14 --cpu-sample 0"
run 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench/trace -o bench -- python3 bench.py $ARGS > gpurun_out/prof_bench/trace.log 2>&1
run 600 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_128B --output-format csv -d gpurun_out/prof_bench/fetch -o bench -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof_bench/fetch.log 2>&1
run 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_bench/write -o bench -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof_bench/write.log 2>&1
# the LDS array that bounds the k = 8 kernel: its busy cycles, conflict
# cycles, atomics, and the clock (GRBM_GUI_ACTIVE / 8 XCDs / duration)
# (the bench's own warm-up, so that the clock has ramped: the last 10 launches are used)
run 600 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_bench/lds -o bench -- python3 bench.py --steps 20 --warmup 14 --cpu-sample 0 > gpurun_out/prof_bench/lds.log 2>&1
tail -1 gpurun_out/prof_bench/trace.log
head -8 gpurun_out/prof_bench/trace/*kernel_stats.csv
