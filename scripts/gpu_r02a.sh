# GPU (round 2, first call): host CPU share probe, full parity suite, default
# bench, and a one-GPU rehearsal of the N-rank bench path (gloo, 2 ranks).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
{ echo "nproc=$(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket"; free -g | head -2; } > gpurun_out/host_probe.txt 2>&1
cat gpurun_out/host_probe.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
grep "^{" gpurun_out/bench.log
KMC_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 3 --cpu-sample -1 > gpurun_out/bench_rehearsal2.log 2>&1 || { tail -5 gpurun_out/bench_rehearsal2.log; exit 1; }
grep "^{" gpurun_out/bench_rehearsal2.log
