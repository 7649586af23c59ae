# GPU: dense parity tests, then the per-rank strong-scaling step cost (scripts/gpu_shard.sh).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_multi.py tests/test_cli.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/dense_tests.log 2>&1; rc=$?
tail -2 gpurun_out/dense_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/dense_tests.log | head -20; exit $rc; fi
bash scripts/gpu_shard.sh
