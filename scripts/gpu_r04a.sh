# GPU (round 4, first run): the tests touched by this round's hygiene changes
# (diag library, spill status flag, cached multi-device state, canonical unaligned /
# caller workspace / big K4s instance, full-size C2/C3), the dense GPU suite, then
# the profile refresh of the bench command: rocprofv3 kernel trace + HBM PMC
# (profile_bench.sh) and the bench line.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04a && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
run 900 $PT tests/test_hash_gpu.py -k "unaligned or big_lists" > $O/tests_new.log 2>&1 || { tail -40 $O/tests_new.log; exit 1; }
tail -3 $O/tests_new.log
run 300 $PT tests/test_abi.py > $O/tests_abi.log 2>&1 || { tail -30 $O/tests_abi.log; exit 1; }
tail -1 $O/tests_abi.log
run 900 $PT -m gpu tests/test_dense_gpu.py > $O/tests_dense.log 2>&1 || { tail -30 $O/tests_dense.log; exit 1; }
tail -2 $O/tests_dense.log
bash scripts/profile_bench.sh || exit $?
run 600 python bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-300
