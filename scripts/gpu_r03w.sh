# GPU (round 3): sampled R4 with non-temporal entry loads and/or eight 16-byte
# loads in flight per lane (variants built from a patched copy outside the tree),
# parity of the combined variant, C3's R4 against the shipped build.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03w && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
KMC_LIB=$V/libkmc_r4abl_nt_u8.so run 300 python -u -m pytest tests/test_dense_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "radix" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in shipped nt u8 nt_u8; do
    if [ $v = shipped ]; then L=""; else L=$V/libkmc_r4abl_$v.so; fi
    KMC_LIB=$L run 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/kbench.py --ks 13 --iters 4 > $O/$v$r.log 2>&1
    echo "== $v $r"; python3 scripts/trace_calls.py $O/$v$r place 3 | grep -E "hist_kernel<13, true|call:" | tail -2
  done
done
