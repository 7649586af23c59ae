# GPU (round 3, final F, the shipped build after the non-temporal sampled R4 loads):
# every GPU test + smoke, the bench line, C1/C3/C3R/C4/C4R with parity checks, the
# fuzzers, and C3's R4 same-box against r03p (plain loads).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03x && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
run 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit 1; }
tail -1 $O/gpu_tests.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
run 600 python bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-250
run 600 python -u scripts/fuzz_dense.py --cases 30 --seed 82 --sampled > $O/fuzz_dense_sampled.log 2>&1
tail -1 $O/fuzz_dense_sampled.log
run 600 python -u scripts/fuzz_dense.py --cases 30 --seed 81 > $O/fuzz_dense.log 2>&1
tail -1 $O/fuzz_dense.log
run 900 python3 scripts/cbench.py --iters 3 > $O/cb.log 2>&1
grep '^{' $O/cb.log | cut -c1-200
for r in 1 2; do
  for v in new old; do
    if [ $v = new ]; then L=""; else L=$V/libkmc_r03p.so; fi
    KMC_LIB=$L run 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/kbench.py --ks 13 --iters 4 > $O/$v$r.log 2>&1
    echo "== $v $r"; python3 scripts/trace_calls.py $O/$v$r place 3 | grep -E "hist_kernel<13, true|call:" | tail -2
  done
done
