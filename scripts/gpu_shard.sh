# GPU: per-rank step cost of the N-way strong-scaling job (scripts/shardbench.py),
# plus the same under a kernel trace for the per-kernel split at N = 8.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/shard && mkdir -p $O && rm -rf $O/*
timeout -k 10 300 python scripts/shardbench.py --worlds ${WORLDS:-1,2,4,8} > $O/shard.log 2>&1 || { tail -5 $O/shard.log; exit 1; }
grep '^{' $O/shard.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o tr -- python3 scripts/shardbench.py --worlds 8 --steps 10 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/shard/tr/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").replace("kmc::", "")
    if "at::" in n or "rocclr" in n: continue
    print("%-60s %5s %10.1f us avg" % (n[:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
