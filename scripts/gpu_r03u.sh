# GPU (round 3): the long-list sampled test on the shipped build, then what bounds
# R4: C3's pipeline (kbench k = 13, 10 Gbase) under rocprofv3 with the shipped
# library and two timing-only ablations of R4 (wrong counts by construction, built
# from a patched copy outside the tree): no LDS adds / no entry loads.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03u && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
run 300 python -u -m pytest tests/test_dense_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "long_list or sampled" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in shipped noadd noload; do
    if [ $v = shipped ]; then L=""; else L=$V/libkmc_r4abl_$v.so; fi
    KMC_LIB=$L run 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/kbench.py --ks 13 --iters 4 > $O/$v$r.log 2>&1
    echo "== $v $r"; python3 scripts/trace_calls.py $O/$v$r place 3 | grep -E "ring|hist|count|place|call:" | grep -v "false>" | tail -6
  done
done
