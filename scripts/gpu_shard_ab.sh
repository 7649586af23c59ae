# GPU: dense parity tests, then scripts/shardbench.py (N = 1 and 8) for the default
# build and lib/variants/libkmc_old.so, alternating.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/shab && mkdir -p $O && rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in default old; do
    L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so; [ $v = old ] && L=$PWD/dna-kmeres-parallel_amd/lib/variants/libkmc_old.so
    KMC_LIB=$L timeout -k 10 300 python scripts/shardbench.py --worlds ${WORLDS:-8,1} --ranks first > $O/$v$r.log 2>&1 || { tail -3 $O/$v$r.log; exit 1; }
    grep '^{' $O/$v$r.log | python3 -c "import sys,json; [print('$v w=%d r=%d step %.4f kernel %.4f' % (d['world'], d['rank'], d['step_ms'], d['kernel_ms'])) for d in map(json.loads, sys.stdin)]"
  done
done
