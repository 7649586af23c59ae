# GPU: canonical parity tests, then C4 under a rocprofv3 kernel trace for the
# default build and every variant build; per-kernel averages of the canon_* kernels.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/c4t && rm -rf gpurun_out/c4t/*
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -m pytest tests/test_hash_gpu.py -q -x -p no:cacheprovider > gpurun_out/c4t/tests.log 2>&1 || { tail -30 gpurun_out/c4t/tests.log; exit 1; }
  tail -1 gpurun_out/c4t/tests.log
fi
one() {  # name lib
  d=gpurun_out/c4t/$1
  KMC_LIB=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o t -- python3 scripts/cbench.py --configs ${CONFIGS:-c4} --iters 3 --cpu-sample-c4 0 --cpu-sample-c3 0 ${CB_ARGS:-} > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  grep '^{' $d.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$1 s_min %.4f s_med %.4f distinct %d' % (d['s_min'], d['s_med'], d.get('distinct', -1)))"
  python3 - $d <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("kmc::", "")
    if "canon" in n or "scan_" in n or "radix" in n:
        print("   %-40s %5s %10.3f ms avg" % (n[:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
}
one default "" || exit 1
for f in dna-kmeres-parallel_amd/lib/variants/*.so; do [ -e "$f" ] && [ -z "$VAR_SKIP" ] || continue
  one $(basename $f .so) $PWD/$f || exit 1
done
