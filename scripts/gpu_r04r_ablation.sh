# GPU (round 4, diagnostic): timing-only ablations of K4s (wrong counts by
# construction, so cbench's checks fail after the timed calls): ablnd skips the
# shared-slot pairwise check, ablnh the crowded-slot rounds; ablbase = the same
# build with neither.  C4 then C4R, under the kernel trace.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04r && mkdir -p $O && rm -rf $O/*
V=$PWD/dna-kmeres-parallel_amd/lib/variants
for v in ablbase ablnd ablnh; do
  KMC_LIB=$V/libkmc_$v.so timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o t -- python3 scripts/cbench.py --configs c4,c4r --iters 3 --cpu-sample-c4 0 > $O/$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"
  case $rc in 124|134|137|139) echo "stopping: rc=$rc"; exit $rc;; esac
  python3 scripts/trace_kernels.py $O/$v canon_sort
done
