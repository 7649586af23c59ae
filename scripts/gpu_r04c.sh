# GPU (round 4): C3 PMC passes (shipped build), a traced cbench of C3 / C4 / C4R
# (rocprofv3 kernel trace: per-kernel times, every result parity-checked by cbench),
# the C4 SQ/LDS PMC groups of the canonical kernels, and the shard steps.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04c && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
if [ -n "$TESTS" ]; then
  run 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu ${TFILES:-tests/test_dense_gpu.py tests/test_baseline_configs_gpu.py} -k "$TESTS" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
run 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cb -o cb -- python3 scripts/cbench.py --iters 3 --configs ${CB:-c3,c4,c4r} > $O/cb.log 2>&1
grep '^{' $O/cb.log | cut -c1-160
python3 scripts/trace_kernels.py $O/cb | tee $O/cb_kernels.txt
if [ -n "$PMC3" ]; then
  KS=13 PMC_OUT=r04c/pmc_c3 run 600 bash scripts/gpu_pmc_c3.sh > $O/pmc_c3.txt 2>&1
fi
if [ -n "$PMC4" ]; then
  run 900 bash scripts/gpu_pmc_c4.sh > $O/pmc_c4.txt 2>&1
fi
if [ -n "$SHARD" ]; then
  run 600 python3 scripts/shardbench.py > $O/shard.log 2>&1
  tail -8 $O/shard.log
fi
