# GPU (round 3, final B): C1 / C3 / C3R / C4 / C4R with their parity checks and CPU
# baselines, the per-rank strong-scaling step costs, the 2-rank gloo rehearsal.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03fb && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 900 python3 scripts/cbench.py --iters 3 > $O/cb.log 2>&1
grep '^{' $O/cb.log | cut -c1-240
run 300 python scripts/shardbench.py --worlds 1,1,2,4,8 > $O/shard.log 2>&1
grep '^{' $O/shard.log | cut -c1-200
KMC_BENCH_BACKEND=gloo run 600 python bench.py --gpus 2 --steps 5 --warmup 3 --cpu-sample 2000000 > $O/bench_gloo2.log 2>&1
grep "^{" $O/bench_gloo2.log | cut -c1-200
