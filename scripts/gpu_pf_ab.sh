# GPU: dense parity tests on the default build, then kernel times for k = 1..8 and C3
# (k = 13) for the default build and lib/variants/libkmc_old.so, alternating.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/pfab && mkdir -p $O && rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in default old; do
    L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so; [ $v = old ] && L=$PWD/dna-kmeres-parallel_amd/lib/variants/libkmc_old.so
    KMC_LIB=$L timeout -k 10 200 python3 scripts/kbench.py --ks 1,4,6,7,8 --iters 15 --tag $v >> $O/kb.log 2>&1 || { tail -3 $O/kb.log; exit 1; }
    KMC_LIB=$L timeout -k 10 300 python3 scripts/cbench.py --configs c3 --iters 3 --no-check --cpu-sample-c3 0 > $O/c3_$v$r.log 2>&1 || { tail -3 $O/c3_$v$r.log; exit 1; }
    grep '^{' $O/c3_$v$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v C3 %.2f ms' % (d['s_med']*1e3))"
  done
done
grep '^{' $O/kb.log | python3 -c "import sys,json; [print('%-8s k=%d %.4f ms' % (d['lib'], d['k'], d['ms_med'])) for d in map(json.loads, sys.stdin)]"
