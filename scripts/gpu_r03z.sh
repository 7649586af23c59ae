# GPU (round 3): non-temporal loads on the exact R4 walk (C3R) and on R5's stage
# reads (C3), variants from scripts/build_r4_ablations.py (R4ABL_REV=HEAD), against
# the shipped build; cbench parity checks on.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03z && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
for r in 1 2; do
  for v in shipped exact_nt place_nt; do
    if [ $v = shipped ]; then L=""; else L=$V/libkmc_r4abl_$v.so; fi
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/cbench.py --configs c3,c3r --iters 3 --cpu-sample-c3 0 > $O/$v$r.log 2>&1
    echo "== $v $r"; grep -h '^{' $O/$v$r.log | cut -c1-100; python3 scripts/trace_calls.py $O/$v$r place 4 | grep -E "hist_kernel|place|call:" | tail -12
  done
done
