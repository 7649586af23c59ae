# GPU box steps, chained: the one parameterised entry for `gpurun` (replaces the
# round-by-round one-off scripts, which live on in git history).
#   usage: bash scripts/gpu_run.sh TAG STEP [STEP ...]
#   steps: tests[:EXPR]   pytest -m gpu (EXPR: a -k expression)
#          abi            the CPU ABI tests in a process of their own (no torch first)
#          smoke          __graft_entry__.smoke()
#          bench          python bench.py (the default line; bench5: the driver's own --warmup 5)
#          rehearsal      bench.py --gpus 2 with gloo, both ranks on the one GPU (strong, then weak): the
#                         N > 1 line's fields, not a measurement
#          profile        scripts/profile_bench.sh: kernel trace + HBM and LDS PMC passes
#          cbench[:CFGS]  scripts/cbench.py --configs CFGS (default c1,c3,c4,c4r) under the kernel trace
#          shard          scripts/shardbench.py (one rank's step of an N-way job, N = 1, 2, 4, 8)
#          pmcshards      scripts/pmc_shards.py run under the FETCH_SIZE and WRITE_SIZE passes (then
#                         `pmc_shards.py parse` here -> profiles/pmc_dense_k8_shards.json)
#          fuzz           the dense and canonical fuzzers
# Every step has its own time limit; the first failing step ends the call.
# Output: gpurun_out/TAG/<step>.log (+ rocprofv3 directories).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG && mkdir -p $O
run() {  # run LIMIT LOG CMD...: stop the whole call on failure
    local lim=$1 log=$2; shift 2
    timeout -k 10 $lim "$@" > $log 2>&1; local rc=$?
    echo "[$(basename $log .log)] rc=$rc"; tail -3 $log
    if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED|Killed" $log | head -20; exit $rc; fi
}
PYT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
for s in "$@"; do
    case $s in
        tests) run 1100 $O/tests.log $PYT tests -m gpu --durations=15 ;;
        tests:*) run 900 $O/tests.log $PYT tests -m gpu -k "${s#tests:}" ;;
        abi) run 300 $O/abi.log $PYT tests/test_abi.py ;;
        smoke) run 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run 600 $O/bench.log python bench.py; grep '^{' $O/bench.log > $O/bench.json ;;
        bench5) run 600 $O/bench5.log python bench.py --gpus 1 --steps 20 --warmup 5; grep '^{' $O/bench5.log > $O/bench5.json ;;
        rehearsal) run 600 $O/rehearsal_strong.log env KMC_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2 &&
                   run 600 $O/rehearsal_weak.log env KMC_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2 --scaling weak --records 2 ;;
        profile) run 1100 $O/profile.log bash scripts/profile_bench.sh ;;
        cbench) run 900 $O/cbench.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/cbench_prof -o cb \
                    -- python3 scripts/cbench.py --iters 3 ;;
        cbench:*) run 900 $O/cbench.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/cbench_prof -o cb \
                      -- python3 scripts/cbench.py --iters 3 --configs "${s#cbench:}" ;;
        shard) run 600 $O/shard.log python scripts/shardbench.py ;;
        pmcshards) run 600 $O/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_128B --output-format csv \
                       -d $O/pmc_fetch -o ps -- python3 scripts/pmc_shards.py run &&
                   run 600 $O/pmc_write.log rocprofv3 --pmc WRITE_SIZE --output-format csv \
                       -d $O/pmc_write -o ps -- python3 scripts/pmc_shards.py run ;;
        fuzz) run 600 $O/fuzz_dense.log python scripts/fuzz_dense.py && run 600 $O/fuzz_canonical.log python scripts/fuzz_canonical.py ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
