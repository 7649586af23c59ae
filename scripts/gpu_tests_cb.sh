# GPU: full parity suite, then configs C3/C4 (scripts/gpu_cbench.sh)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED|Timeout" gpurun_out/gpu_tests.log | head -30; exit $rc; fi
bash scripts/gpu_cbench.sh
