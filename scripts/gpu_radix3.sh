# GPU: radix-path parity (default build), C3 under a kernel trace, then C3 (with
# its parity check) for every diagnostic build in lib/variants/.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${RADIX_OUT:-radix3} && mkdir -p $O && rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "${TK:-radix or golden or many or shards or bench_rank}" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cb -o cb -- python3 scripts/cbench.py --configs c3 --iters 5 --cpu-sample-c3 0 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
grep '^{' $O/cb.log | cut -c1-220
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/*/cb/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("kmc::", "")
    if "at::" in n or "rocprim" in n or "rocclr" in n: continue
    print("%-60s %5s %10.3f ms avg %10.3f max" % (n[:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["MaxNs"]) / 1e6))
PY
for f in dna-kmeres-parallel_amd/lib/variants/${VAR_GLOB:-*}.so; do [ -e "$f" ] || continue
  v=$(basename $f .so); echo "== $v"
  KMC_LIB=$PWD/$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o cb -- python3 scripts/cbench.py --configs c3 --iters 5 --cpu-sample-c3 0 ${VARARGS:-} > $O/var.log 2>&1 || { tail -5 $O/var.log; exit 1; }
  grep '^{' $O/var.log | cut -c1-150
  python3 - $O/$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("kmc::", "")
    if "radix" in n: print("   %-50s %10.3f ms avg" % (n[:50], float(r["AverageNs"]) / 1e6))
PY
done
