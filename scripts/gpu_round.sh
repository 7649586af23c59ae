# GPU: parity tests, kernel micro-bench, bench profile (trace + PMC), then the default bench.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python scripts/kbench.py --ks ${KS:-1,3,4,5,6,7,8} > gpurun_out/kbench.log 2>&1 || exit $?
for f in dna-kmeres-parallel_amd/lib/variants/*.so; do [ -e "$f" ] || continue; KMC_LIB=$PWD/$f timeout -k 10 200 python scripts/kbench.py --ks ${VKS:-5,6} >> gpurun_out/kbench.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/kbench.log | python3 -c "import sys,json; [print('%-22s k=%d %7.3f ms %7.0f GB/s %.3f' % (d['lib'], d['k'], d['ms_med'], d['GBps'], d['frac8TB'])) for d in map(json.loads, sys.stdin)]"
bash scripts/profile_bench.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
grep "^{" gpurun_out/bench.log
