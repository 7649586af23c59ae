# GPU (round 3): the dense kernel with dynamic chunk claims + thieves — parity
# first (dense tests incl. the work-stealing ones), then a same-box A/B against the
# pre-stealing r03a dense kernel (lib/variants/libkmc_r03a.so): kernel times k = 3, 7, 8,
# the concurrent-kernel experiment, per-rank steps; then the whole suite and bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03c && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
OLD=$PWD/dna-kmeres-parallel_amd/lib/variants/libkmc_r03a.so
run 400 python -u -m pytest tests/test_dense_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > $O/dense_tests.log 2>&1 || { grep -E "Error|assert|FAILED|Timeout" $O/dense_tests.log | head -20; tail -5 $O/dense_tests.log; exit 1; }
tail -1 $O/dense_tests.log
for rep in 1 2; do
  run 200 python scripts/kbench.py --ks 3,7,8 --iters 15 >> $O/kbench.log 2>&1
  KMC_LIB=$OLD run 200 python scripts/kbench.py --ks 3,7,8 --iters 15 >> $O/kbench.log 2>&1
done
grep "^{" $O/kbench.log | cut -c1-160
run 300 python scripts/interfere.py --nwgs 0,8,32 > $O/interfere_new.log 2>&1
KMC_LIB=$OLD run 300 python scripts/interfere.py --nwgs 0,8,32 > $O/interfere_old.log 2>&1
echo new; grep "^{" $O/interfere_new.log | cut -c1-160
echo old; grep "^{" $O/interfere_old.log | cut -c1-160
run 300 python scripts/shardbench.py --worlds 1,1,2,4,8 > $O/shard_new.log 2>&1
KMC_LIB=$OLD run 300 python scripts/shardbench.py --worlds 1,1,2,4,8 > $O/shard_old.log 2>&1
echo new; grep '^{' $O/shard_new.log | cut -c1-160
echo old; grep '^{' $O/shard_old.log | cut -c1-160
run 600 python bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-200
run 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit 1; }
tail -1 $O/gpu_tests.log
