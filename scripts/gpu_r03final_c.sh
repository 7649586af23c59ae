# GPU (round 3, final C, after the fmix62 lists and the last tests): full parity suite
# + smoke, the bench line, the dense fuzzer (exact and sampled radix modes) and the
# canonical fuzzer.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03fc && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit 1; }
tail -1 $O/gpu_tests.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
run 600 python bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-250
run 600 python -u scripts/fuzz_dense.py --cases 40 --seed 31 > $O/fuzz_dense.log 2>&1
tail -1 $O/fuzz_dense.log
run 600 python -u scripts/fuzz_dense.py --cases 30 --seed 32 --sampled > $O/fuzz_dense_sampled.log 2>&1
tail -1 $O/fuzz_dense_sampled.log
run 600 python -u scripts/fuzz_canonical.py > $O/fuzz_canonical.log 2>&1
tail -1 $O/fuzz_canonical.log
