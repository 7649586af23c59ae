# GPU: per-phase clock profile of the R3 ring kernel (workgroup 0) for every
# diagnostic build in lib/variants/ (KMC_RING_PROF=1 builds print ring_prof lines).
cd $GRAFT_REPO_ROOT && O=gpurun_out/ringprof && mkdir -p $O && rm -rf $O/*
for f in dna-kmeres-parallel_amd/lib/variants/${RP_GLOB:-*}.so; do [ -e "$f" ] || continue
  v=$(basename $f .so); echo "== $v"
  KMC_LIB=$PWD/$f timeout -k 10 300 python3 scripts/cbench.py --configs c3 --iters 1 --cpu-sample-c3 0 --no-check > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  grep '^{' $O/$v.log | cut -c1-150
  grep ring_prof $O/$v.log | awk 'NR<=16'
done
