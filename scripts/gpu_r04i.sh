# GPU (round 4, profiles of the shipped build): the bench command's kernel trace +
# HBM PMC (profile_bench.sh) and the bench line; C1 / C3 / C4 / C4R through
# scripts/cbench.py under the kernel trace (every result parity-checked); then C4
# against lib/variants/libkmc_k3base.so (the canonical source before this round),
# same box, alternating.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04i && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
bash scripts/profile_bench.sh > $O/profile_bench.txt 2>&1 || { tail -20 $O/profile_bench.txt; exit 1; }
tail -12 $O/profile_bench.txt
run 600 python3 bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log | cut -c1-600
run 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cb -o cb -- python3 scripts/cbench.py --iters 3 --configs c1,c3,c4,c4r > $O/cb.log 2>&1
grep '^{' $O/cb.log | cut -c1-220
python3 scripts/trace_kernels.py $O/cb > $O/cb_kernels.txt; grep -E "canon_|radix_|count_dense|reduce_dense" $O/cb_kernels.txt
V=$PWD/dna-kmeres-parallel_amd/lib/variants
for r in 1 2; do
  for v in k3base new; do
    L=$V/libkmc_$v.so; [ $v = new ] && L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/cbench.py --configs c4 --iters 3 --cpu-sample-c4 0 > $O/$v$r.log 2>&1
    echo "== $v $r $(grep -o '"s_med": [0-9.]*' $O/$v$r.log | tr '\n' ' ')"; python3 scripts/trace_kernels.py $O/$v$r canon_
  done
done
