# GPU (round 4): R3 flush variants of the radix path (scripts/build_src_variants.sh:
# base, circular ring, predicated flush reads, both), timed same-box in alternating
# order on C3's 10 Gbase k = 13 pipeline (kbench under rocprofv3 kernel trace),
# then the radix parity tests on the variant VARIANT_TEST (KMC_LIB + KMC_DIAG_LIB),
# then the C3 PMC passes of the shipped build.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04b && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
for r in 1 2; do
  for v in ${VARIANTS:-base circ pred cp}; do
    KMC_LIB=$V/libkmc_$v.so run 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/kbench.py --ks 13 --iters 5 > $O/$v$r.log 2>&1
    echo "== $v $r $(grep -o '"ms_med": [0-9.]*' $O/$v$r.log)"; python3 scripts/trace_kernels.py $O/$v$r radix_ | grep -E "ring|hist|count|place"
  done
done
if [ -n "$VARIANT_TEST" ]; then
  KMC_LIB=$V/libkmc_$VARIANT_TEST.so KMC_DIAG_LIB=$V/libkmc_${VARIANT_TEST}_diag.so run 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_dense_gpu.py -k "radix or k13 or 13" > $O/tests_$VARIANT_TEST.log 2>&1 || { tail -30 $O/tests_$VARIANT_TEST.log; exit 1; }
  tail -2 $O/tests_$VARIANT_TEST.log
fi
if [ -n "$PMC" ]; then
  KS=13 PMC_OUT=r04b/pmc_c3 run 600 bash scripts/gpu_pmc_c3.sh > $O/pmc_c3.txt 2>&1
  grep -A30 "ring_kernel" $O/pmc_c3.txt | head -40
fi
