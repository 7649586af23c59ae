# GPU: parity tests on the default build, then kbench over every variant build.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
run() { timeout -k 10 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
fi
: > gpurun_out/kbench.log
run 200 python scripts/kbench.py --ks ${KS:-3,7,8} >> gpurun_out/kbench.log 2>&1
for f in dna-kmeres-parallel_amd/lib/variants/*.so; do
  KMC_LIB=$PWD/$f run 200 python scripts/kbench.py --ks ${KS:-3,7,8} >> gpurun_out/kbench.log 2>&1
done
grep -v amdgpu.ids gpurun_out/kbench.log | python3 -c "import sys,json; [print('%-22s k=%d %7.3f ms %7.0f GB/s %.3f' % (d['lib'], d['k'], d['ms_med'], d['GBps'], d['frac8TB'])) for d in map(json.loads, sys.stdin)]"
