# GPU (round 4, final build): the bench command's kernel trace + HBM PMC
# (profile_bench.sh), the bench line at N = 1, and one rank's step of an N-way
# job at N = 1, 2, 4, 8 (shardbench) -- profiles of HEAD for the dense path.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04ai && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
bash scripts/profile_bench.sh > $O/profile_bench.txt 2>&1 || { tail -20 $O/profile_bench.txt; exit 1; }
tail -12 $O/profile_bench.txt
run 600 python3 bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-700
run 300 python3 scripts/shardbench.py --worlds 1,2,4,8 > $O/shard.log 2>&1
grep '^{' $O/shard.log | cut -c1-170
