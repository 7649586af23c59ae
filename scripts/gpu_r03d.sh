# GPU (round 3): parity of the dense work-stealing kernel and the circular-ring R3
# (test_dense_gpu.py: k = 1..13), then same-box A/B against the r03a build
# (lib/variants/libkmc_r03a.so: static home ranges, tail-moving rings): dense kernel
# times, the concurrent-kernel experiment, per-rank steps, C3 with per-kernel times.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03d && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
OLD=$PWD/dna-kmeres-parallel_amd/lib/variants/libkmc_r03a.so
run 400 python -u -m pytest tests/test_dense_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > $O/dense_tests.log 2>&1
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
for r in 1 2; do
  for v in new old; do
    L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so; [ $v = old ] && L=$OLD
    KMC_LIB=$L run 300 rocprofv3 --kernel-trace --output-format csv -d $O/c3_$v$r -o t -- python3 scripts/cbench.py --configs c3 --iters 3 --cpu-sample-c3 0 > $O/c3_$v$r.log 2>&1
    echo "== C3 $v ($r)"; grep '^{' $O/c3_$v$r.log | cut -c1-200
    python3 scripts/trace_kernels.py $O/c3_$v$r radix
  done
done
