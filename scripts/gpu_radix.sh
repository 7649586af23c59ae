# GPU: radix-path parity tests (k = 9..13), then C3 timing for the default build and variants.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "${TK:-9 or 10 or 11 or 12 or 13 or radix or shard}" > gpurun_out/radix_tests.log 2>&1; rc=$?
tail -3 gpurun_out/radix_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/radix_tests.log | head -20; exit $rc; fi
: > gpurun_out/c3.log
timeout -k 10 300 python scripts/cbench.py --configs c3 --iters 5 >> gpurun_out/c3.log 2>&1 || exit $?
for f in dna-kmeres-parallel_amd/lib/variants/*.so; do [ -e "$f" ] || continue; echo "$f" >> gpurun_out/c3.log; KMC_LIB=$PWD/$f timeout -k 10 300 python scripts/cbench.py --configs c3 --iters 5 >> gpurun_out/c3.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/c3.log
