# GPU (round 2, re-entry): full parity suite + smoke, the default bench line, and the
# bench under a kernel trace + HBM PMC (scripts/profile_bench.sh).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r02c && mkdir -p $O && rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep "^{" $O/bench.log
bash scripts/profile_bench.sh || exit $?
