# GPU (round 3): canonical counting (C4 / C4R, cbench parity checks on) with
# non-temporal entry loads in K3b and/or K4s (scripts/build_hash_variants.py)
# against the shipped build, per-call kernel times.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03y && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
for r in 1 2; do
  for v in shipped fine_nt sort_nt both_nt; do
    if [ $v = shipped ]; then L=""; else L=$V/libkmc_hash_$v.so; fi
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/cbench.py --configs c4,c4r --iters 2 > $O/$v$r.log 2>&1
    echo "== $v $r"; grep -h '^{' $O/$v$r.log | cut -c1-60; python3 scripts/trace_calls.py $O/$v$r place 6 | grep -E "fine|sort_k|call:" | grep -B0 -A0 "" | tail -9
  done
done
