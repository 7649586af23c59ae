# GPU (round 4, validation of the shipped build): the whole -m gpu suite (test_abi in
# its own process: it may initialise HIP before torch), smoke(), the dense / sampled
# radix / canonical fuzzers, then the bench command's kernel trace + HBM PMC
# (profile_bench.sh) and the bench line.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04h && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
if [ -z "$NOTESTS" ]; then
run 1100 $PT -m gpu tests --ignore=tests/test_abi.py > $O/tests_gpu.log 2>&1 || { tail -30 $O/tests_gpu.log; exit 1; }
tail -1 $O/tests_gpu.log
run 300 $PT tests/test_abi.py > $O/tests_abi.log 2>&1 || { tail -30 $O/tests_abi.log; exit 1; }
tail -1 $O/tests_abi.log
run 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
if [ -n "$FUZZ" ]; then
run 600 python3 scripts/fuzz_dense.py > $O/fuzz_dense.log 2>&1 || { tail -20 $O/fuzz_dense.log; exit 1; }
tail -1 $O/fuzz_dense.log
run 600 python3 scripts/fuzz_canonical.py > $O/fuzz_canonical.log 2>&1 || { tail -20 $O/fuzz_canonical.log; exit 1; }
tail -1 $O/fuzz_canonical.log
fi
if [ -n "$PROF" ]; then
bash scripts/profile_bench.sh > $O/profile_bench.txt 2>&1 || { tail -20 $O/profile_bench.txt; exit 1; }
tail -10 $O/profile_bench.txt
run 600 python3 bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-400
fi
