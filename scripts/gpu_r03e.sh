# GPU (round 3): what the dense kernel's chunk claims cost (same box): current build,
# thieves off, 128- and 512-tile claims, the r03a static build; the concurrent-kernel
# experiment; C3 with the circular-ring R3 against r03a, per-kernel times.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03e && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
for rep in 1 2; do
  run 200 python scripts/kbench.py --ks 3,8 --iters 12 >> $O/kbench.log 2>&1
  KMC_NO_STEAL=1 run 200 python scripts/kbench.py --ks 3,8 --iters 12 --tag nosteal >> $O/kbench.log 2>&1
  for v in chunk128 chunk512 r03a; do KMC_LIB=$V/libkmc_$v.so run 200 python scripts/kbench.py --ks 3,8 --iters 12 >> $O/kbench.log 2>&1; done
done
grep "^{" $O/kbench.log | python3 -c "import sys,json; [print('%-40s k=%d %.3f ms' % (d['lib'][-40:], d['k'], d['ms_med'])) for d in map(json.loads, sys.stdin)]"
for v in new chunk512 r03a; do
  L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so; [ $v != new ] && L=$V/libkmc_$v.so
  KMC_LIB=$L run 300 python scripts/interfere.py --nwgs 0,8,32 > $O/interfere_$v.log 2>&1
  echo "== interfere $v"; grep "^{" $O/interfere_$v.log | cut -c1-150
done
for r in 1 2; do
  for v in new old; do
    L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so; [ $v = old ] && L=$V/libkmc_r03a.so
    KMC_LIB=$L run 300 rocprofv3 --kernel-trace --output-format csv -d $O/c3_$v$r -o t -- python3 scripts/cbench.py --configs c3 --iters 3 --cpu-sample-c3 0 > $O/c3_$v$r.log 2>&1
    echo "== C3 $v ($r)"; grep '^{' $O/c3_$v$r.log | cut -c1-220
    python3 scripts/trace_kernels.py $O/c3_$v$r radix
  done
done
