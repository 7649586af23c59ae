# GPU (round 4, validation of the final build after the K4s crowded-slot rewrite): the whole -m gpu suite,
# test_abi, smoke(), the dense and canonical fuzzers (scripts/gpu_r04h.sh, FUZZ=1);
# then C1 / C3 / C4 / C4R through scripts/cbench.py under the kernel trace (every
# result parity-checked) and the SQ / HBM counters of the C4 kernels
# (scripts/gpu_pmc_c4.sh).  The dense bench path is unchanged since r04o.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04ah && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
FUZZ=1 bash scripts/gpu_r04h.sh || exit 1
run 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cb -o cb -- python3 scripts/cbench.py --iters 3 --configs c1,c3,c4,c4r > $O/cb.log 2>&1
grep '^{' $O/cb.log | cut -c1-260
python3 scripts/trace_kernels.py $O/cb > $O/cb_kernels.txt; grep -E "canon_|radix_" $O/cb_kernels.txt
bash scripts/gpu_pmc_c4.sh > $O/pmc4.log 2>&1 || { tail -5 $O/pmc4.log; exit 1; }
echo pmc done
