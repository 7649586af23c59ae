# GPU (round 3): canonical lists of fmix62 values (the unmix moves from K4s / K4 to
# the place kernel): canonical parity tests, then C4 / C4R same-box against r03a
# with per-call kernel times.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03m && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
run 600 python -u -m pytest tests/test_hash_gpu.py tests/test_cli.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in new old; do
    L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so; [ $v = old ] && L=$V/libkmc_r03a.so
    KMC_LIB=$L run 500 rocprofv3 --kernel-trace --output-format csv -d $O/cb_$v$r -o t -- python3 scripts/cbench.py --configs c4,c4r --iters 2 --cpu-sample-c4 0 > $O/cb_$v$r.log 2>&1
    echo "== $v ($r)"; grep -h '^{' $O/cb_$v$r.log | cut -c1-100
    if [ $r = 1 ]; then python3 scripts/trace_calls.py $O/cb_$v$r recoff 4 | grep -E "call|canon" | grep -v "0.0[0-9][0-9] ms"; fi
  done
done
