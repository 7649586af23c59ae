# GPU (round 2, final after the walk prefetch): full parity suite + smoke, the default bench line, the bench
# under rocprofv3 (kernel trace + HBM PMC: scripts/profile_bench.sh), C3/C4/C4R with
# their parity checks, and the per-rank strong-scaling step cost.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r02h && mkdir -p $O && rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep "^{" $O/bench.log | cut -c1-200
bash scripts/profile_bench.sh > $O/profile_bench.log 2>&1 || { tail -5 $O/profile_bench.log; exit 1; }
timeout -k 10 900 python3 scripts/cbench.py --iters 3 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
grep '^{' $O/cb.log | cut -c1-240
timeout -k 10 300 python scripts/shardbench.py > $O/shard.log 2>&1 || { tail -5 $O/shard.log; exit 1; }
grep '^{' $O/shard.log | cut -c1-200
