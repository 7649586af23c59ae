# GPU (round 4): same-box A/B of this round's walk and launch changes, then parity.
#  1. C4 (cbench, parity-checked): lib/variants/libkmc_k3base.so (canonical walks
#     before the change) against the new build (templated K1 / K3a, branch-free
#     K1 adds and K3a staged round, batched K3a write-out; k4w0: that, with K4s as
#     before; k4b0: + K4s's explicit key wait; plb0: all but the place kernel's
#     batched count loads; new: everything),
#     two alternating rounds;
#  2. one rank's step of an N-way job (shardbench, N = 1 and 8): dvec0 (dense
#     launch as before) against dvec1 (parallel first-record search, 16-byte LDS
#     clear and slab flush), two alternating rounds;
#  3. the canonical, full-size and dense GPU tests on the new build.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04g && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
M=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
if [ -z "$SKIPC4" ]; then
for r in 1 2; do
  for v in ${C4V:-k3base k4w0 k4b0 plb0 new}; do
    L=$V/libkmc_$v.so; [ $v = new ] && L=$M
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/cbench.py --configs c4 --iters 3 --cpu-sample-c4 0 > $O/$v$r.log 2>&1
    echo "== $v $r $(grep -o '"s_med": [0-9.]*' $O/$v$r.log | tr '\n' ' ')"; python3 scripts/trace_kernels.py $O/$v$r canon_
  done
done
fi
for r in 1 2; do
  for v in dvec0 dvec1; do
    KMC_LIB=$V/libkmc_$v.so run 300 python3 scripts/shardbench.py --worlds 1,8 > $O/shard_$v$r.log 2>&1
    echo "== $v $r"; grep '^{' $O/shard_$v$r.log | cut -c1-200
  done
done
run 900 $PT tests/test_hash_gpu.py tests/test_baseline_configs_gpu.py > $O/tests_hash.log 2>&1 || { tail -30 $O/tests_hash.log; exit 1; }
tail -1 $O/tests_hash.log
run 900 $PT tests/test_dense_gpu.py > $O/tests_dense.log 2>&1 || { tail -30 $O/tests_dense.log; exit 1; }
tail -1 $O/tests_dense.log
