# GPU (round 3): C3 (kernel trace) and C3R same-box, sampled radix partition vs r03a.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03g && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
for r in 1 2; do
  for v in new old; do
    L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so; [ $v = old ] && L=$V/libkmc_r03a.so
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/c3_$v$r -o t -- python3 scripts/cbench.py --configs c3 --iters 3 --cpu-sample-c3 0 > $O/c3_$v$r.log 2>&1
    KMC_LIB=$L run 400 python3 scripts/cbench.py --configs c3r --iters 3 > $O/c3r_$v$r.log 2>&1
    echo "== $v ($r)"; grep -h '^{' $O/c3_$v$r.log $O/c3r_$v$r.log | cut -c1-100
    python3 scripts/trace_kernels.py $O/c3_$v$r radix
  done
done
