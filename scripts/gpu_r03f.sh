# GPU (round 3): the sampled radix partition (C3): radix parity tests (exact, sampled,
# forced overflow -> gated exact rerun), then C3 and C3R same-box against r03a with
# per-kernel times.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03f && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
run 400 python -u -m pytest tests/test_dense_gpu.py -q -x -k "radix" -p no:cacheprovider --timeout 200 --timeout-method thread > $O/radix_tests.log 2>&1 || { tail -30 $O/radix_tests.log; exit 1; }
tail -1 $O/radix_tests.log
for r in 1 2; do
  for v in new old; do
    L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so; [ $v = old ] && L=$V/libkmc_r03a.so
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/c3_$v$r -o t -- python3 scripts/cbench.py --configs c3,c3r --iters 3 --cpu-sample-c3 0 > $O/c3_$v$r.log 2>&1
    echo "== $v ($r)"; grep '^{' $O/c3_$v$r.log | cut -c1-120
    python3 scripts/trace_kernels.py $O/c3_$v$r radix
  done
done
