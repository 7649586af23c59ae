# GPU (round 3): sampled radix partition with overflow lists (register-cached R4
# regions): radix parity tests,
# then C3 / C3R same-box against r03a with per-call kernel breakdowns; the
# concurrent-kernel experiment with 0 or 8 CUs left out of the dense grid.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03j && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
run 400 python -u -m pytest tests/test_dense_gpu.py -q -x -k "radix" -p no:cacheprovider --timeout 200 --timeout-method thread > $O/radix_tests.log 2>&1 || { tail -30 $O/radix_tests.log; exit 1; }
tail -1 $O/radix_tests.log
for r in 1 2; do
  for v in new old; do
    L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so; [ $v = old ] && L=$V/libkmc_r03a.so
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/c3_$v$r -o t -- python3 scripts/cbench.py --configs c3,c3r --iters 3 --cpu-sample-c3 0 > $O/c3_$v$r.log 2>&1
    echo "== $v ($r)"; grep -h '^{' $O/c3_$v$r.log | cut -c1-100
    if [ $r = 1 ]; then python3 scripts/trace_calls.py $O/c3_$v$r place 4; fi
  done
done
run 400 python scripts/interfere.py --worlds 1,8 --nwgs 0,8 --reserve 0,8 > $O/interfere.log 2>&1
grep '^{' $O/interfere.log | cut -c1-170
