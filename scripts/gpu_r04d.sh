# GPU (round 4): the vmcnt pre-wait variants (stores counted in vmcnt on gfx9):
# R3 (radix, C3) r3base vs r3pw and K3b (canonical, C4) k3base vs k3pw, same box,
# alternating order, under the kernel trace; then the parity tests on both new
# variants (KMC_LIB + KMC_DIAG_LIB).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04d && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
for r in 1 2; do
  for v in r3base r3pw; do
    KMC_LIB=$V/libkmc_$v.so run 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/kbench.py --ks 13 --iters 5 > $O/$v$r.log 2>&1
    echo "== $v $r $(grep -o '"ms_med": [0-9.]*' $O/$v$r.log)"; python3 scripts/trace_kernels.py $O/$v$r radix_ | grep -E "ring|hist"
  done
  for v in ${K3V:-k3base k3pw k3apw k3both}; do
    KMC_LIB=$V/libkmc_$v.so run 400 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/cbench.py --configs c4 --iters 3 --cpu-sample-c4 0 > $O/$v$r.log 2>&1
    echo "== $v $r $(grep -o '"s_med": [0-9.]*' $O/$v$r.log)"; python3 scripts/trace_kernels.py $O/$v$r canon_
  done
done
KMC_LIB=$V/libkmc_r3pw.so KMC_DIAG_LIB=$V/libkmc_r3pw_diag.so run 600 $PT tests/test_dense_gpu.py -k "radix or 13" > $O/tests_r3pw.log 2>&1 || { tail -20 $O/tests_r3pw.log; exit 1; }
tail -1 $O/tests_r3pw.log
KMC_LIB=$V/libkmc_k3both.so KMC_DIAG_LIB=$V/libkmc_k3both_diag.so run 600 $PT tests/test_hash_gpu.py -k "not repeat_rich" > $O/tests_k3both.log 2>&1 || { tail -20 $O/tests_k3both.log; exit 1; }
tail -1 $O/tests_k3both.log
