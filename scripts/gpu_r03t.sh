# GPU (round 3): sampled R4 walks its lists in chunks (bounds read with v_readlane,
# no region cursor in LDS): dense/radix parity tests (incl. the long-list fallback)
# + exact and sampled fuzz, then C3 / C3R per-call kernel times same-box against r03p.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03t && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
run 600 python -u -m pytest tests/test_dense_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run 600 python -u scripts/fuzz_dense.py --cases 30 --seed 72 --sampled > $O/fuzz_sampled.log 2>&1
tail -1 $O/fuzz_sampled.log
for r in 1 2; do
  run 400 rocprofv3 --kernel-trace --output-format csv -d $O/new$r -o t -- python3 scripts/cbench.py --configs c3 --iters 3 --cpu-sample-c3 0 > $O/new$r.log 2>&1
  KMC_LIB=$V/libkmc_r03p.so run 400 rocprofv3 --kernel-trace --output-format csv -d $O/old$r -o t -- python3 scripts/cbench.py --configs c3 --iters 3 --cpu-sample-c3 0 > $O/old$r.log 2>&1
  for v in new old; do echo "== $v $r"; grep -h '^{' $O/$v$r.log | cut -c1-110; python3 scripts/trace_calls.py $O/$v$r place 4 | grep -E "hist|call:" ; done
done
