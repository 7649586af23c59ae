# GPU (round 4): every remaining wave scan / wave sum as DPP steps (the block scan
# of kmc_scan.h, the sampled R4's region-table scan, the dense launch's wave sums)
# -- new -- against f57 (the whole library at f57ccf8).  Same box, alternating:
# C3 and C4 via cbench under the kernel trace, one rank's step at N = 1 and 8
# (shardbench), then the whole -m gpu suite on the new build.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04z && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
M=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so
for r in 1 2; do
  for v in f57 new; do
    L=$V/libkmc_$v.so; [ $v = new ] && L=$M
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/cbench.py --configs c3,c4 --iters 3 --cpu-sample-c4 0 --cpu-sample-c3 0 > $O/$v$r.log 2>&1
    echo "== $v $r $(grep -o '"s_med": [0-9.]*' $O/$v$r.log | tr '\n' ' ')"; python3 scripts/trace_kernels.py $O/$v$r | grep -E "canon_sort|coarse|radix_hist|radix_ring|scan_"
    KMC_LIB=$L run 300 python3 scripts/shardbench.py --worlds 1,8 > $O/shard_$v$r.log 2>&1
    grep '^{' $O/shard_$v$r.log | cut -c1-160
  done
done
run 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests --ignore=tests/test_abi.py > $O/tests_gpu.log 2>&1 || { tail -30 $O/tests_gpu.log; exit 1; }
tail -1 $O/tests_gpu.log
