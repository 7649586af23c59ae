# GPU: canonical parity (default build), C4/C4R under a kernel trace, then C4 for
# every diagnostic build in lib/variants/ (VAR_GLOB), each under a kernel trace.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
CFGS=${CFGS:-c4,c4r} bash scripts/gpu_c4r.sh || exit 1
for f in dna-kmeres-parallel_amd/lib/variants/${VAR_GLOB:-*}.so; do [ -e "$f" ] || continue
  v=$(basename $f .so); echo "== $v"
  KMC_LIB=$PWD/$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4r/$v -o cb -- python3 scripts/cbench.py --configs ${VCFGS:-c4} --iters 3 --cpu-sample-c4 0 > gpurun_out/c4r/var.log 2>&1 || { tail -5 gpurun_out/c4r/var.log; exit 1; }
  grep '^{' gpurun_out/c4r/var.log | cut -c1-200
  python3 - gpurun_out/c4r/$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("kmc::", "")
    if "canon" in n: print("   %-40s %10.3f ms avg" % (n[:40], float(r["AverageNs"]) / 1e6))
PY
done
