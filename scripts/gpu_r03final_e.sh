# GPU (round 3, final E, the shipped build): C1 / C3 / C3R / C4 / C4R with their
# parity checks and CPU baselines, the per-rank strong-scaling step costs, the
# 2-rank gloo rehearsal of the N > 1 line, and the dense / sampled / canonical fuzzers.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03r && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 900 python3 scripts/cbench.py --iters 3 > $O/cb.log 2>&1
grep '^{' $O/cb.log | cut -c1-240
run 300 python scripts/shardbench.py --worlds 1,1,2,4,8 > $O/shard.log 2>&1
grep '^{' $O/shard.log | cut -c1-200
KMC_BENCH_BACKEND=gloo run 600 python bench.py --gpus 2 --steps 5 --warmup 3 --cpu-sample 2000000 > $O/bench_gloo2.log 2>&1
grep "^{" $O/bench_gloo2.log | cut -c1-200
run 600 python -u scripts/fuzz_dense.py --cases 40 --seed 61 > $O/fuzz_dense.log 2>&1
tail -1 $O/fuzz_dense.log
run 600 python -u scripts/fuzz_dense.py --cases 30 --seed 62 --sampled > $O/fuzz_dense_sampled.log 2>&1
tail -1 $O/fuzz_dense_sampled.log
run 600 python -u scripts/fuzz_canonical.py > $O/fuzz_canonical.log 2>&1
tail -1 $O/fuzz_canonical.log
