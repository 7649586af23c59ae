# GPU: parity tests, then kernel micro-bench for $KS (default lib).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 600 python scripts/kbench.py --ks ${KS:-3,8} > gpurun_out/kbench.log 2>&1 || { tail -5 gpurun_out/kbench.log; exit 1; }
grep "^{" gpurun_out/kbench.log | python3 -c "import sys,json; [print('%-22s k=%d %8.3f ms %7.0f GB/s %.3f' % (d['lib'], d['k'], d['ms_med'], d['GBps'], d['frac8TB'])) for d in map(json.loads, sys.stdin)]"
