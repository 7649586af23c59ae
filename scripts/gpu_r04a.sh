# GPU (round 4, first run): the tests touched by this round's hygiene changes
# (diag library, spill status flag, cached multi-device state, canonical unaligned /
# caller workspace, full-size C2/C3), then the profile refresh of the build:
# rocprofv3 kernel trace + HBM PMC of the bench command (profile_bench.sh), the
# bench line, the C3 sampled-pipeline PMC, a traced C3/C4/C4R cbench, shard steps.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04a && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
run 900 $PT tests/test_abi.py tests/test_baseline_configs_gpu.py "tests/test_dense_gpu.py::test_count_multi_single_device" "tests/test_dense_gpu.py::test_dense_spill_overflow_raises_status" tests/test_hash_gpu.py -k "not repeat_rich" > $O/tests_new.log 2>&1 || { tail -30 $O/tests_new.log; exit 1; }
tail -3 $O/tests_new.log
run 900 $PT -m gpu tests/test_dense_gpu.py > $O/tests_dense.log 2>&1 || { tail -30 $O/tests_dense.log; exit 1; }
tail -2 $O/tests_dense.log
bash scripts/profile_bench.sh || exit $?
run 600 python bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-300
KS=13 PMC_OUT=r04a/pmc_c3 run 600 bash scripts/gpu_pmc_c3.sh > $O/pmc_c3.txt 2>&1
run 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cb -o cb -- python3 scripts/cbench.py --iters 3 --configs c3,c4,c4r > $O/cb.log 2>&1
grep '^{' $O/cb.log | cut -c1-200
run 600 python3 scripts/shardbench.py > $O/shard.log 2>&1
tail -8 $O/shard.log
