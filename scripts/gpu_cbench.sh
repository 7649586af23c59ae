# GPU: configs C3 (k=13 radix) and C4 (k=31 canonical) under a rocprofv3 kernel trace;
# prints the JSON lines and the per-kernel summary.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/cb && rm -rf gpurun_out/cb/*
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cb -o cb -- python3 scripts/cbench.py --iters ${ITERS:-3} ${CB_ARGS} > gpurun_out/cb/log 2>&1 || { tail -20 gpurun_out/cb/log; exit 1; }
grep '^{' gpurun_out/cb/log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/cb/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("kmc::", "")
    print("%-70s %5s %10.3f ms avg %6.2f%%" % (n[:70], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
PY
