# GPU: rocprofv3 kernel trace (stats) of kbench for $KS; prints the per-kernel summary.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ktrace && rm -rf gpurun_out/ktrace/*
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktrace -o kt -- python3 scripts/kbench.py --ks ${KS:-8} --iters ${ITERS:-3} > gpurun_out/ktrace/log 2>&1 || { tail -5 gpurun_out/ktrace/log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ktrace/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("kmc::", "")
    print("%-70s %5s %10.3f ms avg %6.2f%%" % (n[:70], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
PY
