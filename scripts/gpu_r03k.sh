# GPU (round 3 checkpoint): every GPU test, smoke, bench (N = 1) with a rocprofv3
# kernel-trace summary, the 2-rank gloo rehearsal of the N > 1 line (reserved CUs),
# C3 / C3R with per-call kernel times.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03k && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit 1; }
tail -1 $O/gpu_tests.log
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
run 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 bench.py > $O/bench.log 2>&1
grep '^{' $O/bench.log | cut -c1-400
KMC_BENCH_BACKEND=gloo run 400 python bench.py --gpus 2 --steps 5 --warmup 3 > $O/rehearsal.log 2>&1
grep '^{' $O/rehearsal.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d['config'][k] for k in ('rccl_world','backend','reserved_cus','rccl_max_channels')}, d['roofline']['node_frac'], d['allreduce']['ms'])"
run 400 rocprofv3 --kernel-trace --output-format csv -d $O/c3 -o t -- python3 scripts/cbench.py --configs c3,c3r --iters 3 --cpu-sample-c3 0 > $O/c3.log 2>&1
grep -h '^{' $O/c3.log | cut -c1-120
python3 scripts/trace_calls.py $O/c3 place 4 | grep -v fillBuffer
