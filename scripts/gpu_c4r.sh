# GPU: canonical parity tests (incl. the repeat-rich genome), then C4 and C4R with
# their parity checks under a kernel trace.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/c4r && mkdir -p $O && rm -rf $O/*
timeout -k 10 600 python -u -m pytest tests/test_hash_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cb -o cb -- python3 scripts/cbench.py --configs ${CFGS:-c4,c4r} --iters 3 --cpu-sample-c4 0 > $O/cb.log 2>&1 || { tail -20 $O/cb.log; exit 1; }
grep '^{' $O/cb.log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c4r/cb/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("kmc::", "")
    if "at::" in n or "rocprim" in n or "rocclr" in n: continue
    print("%-50s %5s %10.3f ms avg %10.3f max" % (n[:50], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["MaxNs"]) / 1e6))
PY
