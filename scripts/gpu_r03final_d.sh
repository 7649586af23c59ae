# GPU (round 3, final D, after the in-kernel k = 8 recount): full parity suite + smoke, the default bench line, and the
# bench under rocprofv3 (kernel trace + HBM PMC passes: scripts/profile_bench.sh).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03p && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit 1; }
tail -1 $O/gpu_tests.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
run 600 python bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-300
run 1000 bash scripts/profile_bench.sh > $O/profile_bench.log 2>&1
tail -12 $O/profile_bench.log | cut -c1-200
