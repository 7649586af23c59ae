# GPU: dense-path parity (test_dense_gpu, test_dist_gpu, CLI) + the default bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/dense && mkdir -p $O && rm -rf $O/*
timeout -k 10 900 python -u -m pytest tests/test_dense_gpu.py tests/test_cli.py tests/test_multi.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; fi
timeout -k 10 400 python bench.py --cpu-sample -1 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-400
KMC_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 4 --cpu-sample -1 > $O/bench_r2.log 2>&1 || { tail -5 $O/bench_r2.log; exit 1; }
grep '^{' $O/bench_r2.log | cut -c1-300
