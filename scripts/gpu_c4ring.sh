# GPU: canonical parity (default build), C4/C4R under a kernel trace, then C4 for
# every diagnostic build in lib/variants/.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
CFGS=${CFGS:-c4,c4r} bash scripts/gpu_c4r.sh || exit 1
for f in dna-kmeres-parallel_amd/lib/variants/*.so; do [ -e "$f" ] || continue
  echo "== $f"; KMC_LIB=$PWD/$f timeout -k 10 300 python scripts/cbench.py --configs c4 --iters 3 --cpu-sample-c4 0 > gpurun_out/c4r/var.log 2>&1 || { tail -5 gpurun_out/c4r/var.log; exit 1; }
  grep '^{' gpurun_out/c4r/var.log | cut -c1-300
done
