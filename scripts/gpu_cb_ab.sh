# GPU: same-box A/B of C3 and C4 (no checks) for the default build and every
# lib/variants build, alternating, with per-kernel times from a kernel trace.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/cbab && mkdir -p $O && rm -rf $O/*
for r in 1 2; do
  for f in dna-kmeres-parallel_amd/lib/libkmc.so dna-kmeres-parallel_amd/lib/variants/*.so; do
    v=$(basename $f .so)
    KMC_LIB=$PWD/$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/cbench.py --configs ${CFGS:-c3,c4} --iters 2 --no-check --cpu-sample-c3 0 --cpu-sample-c4 0 > $O/$v$r.log 2>&1 || { tail -3 $O/$v$r.log; exit 1; }
    echo "== $v ($r)"; grep '^{' $O/$v$r.log | python3 -c "import sys,json; [print('  %s %.2f ms' % (d['config'], d['s_med']*1e3)) for d in map(json.loads, sys.stdin)]"
    python3 - $O/$v$r <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("kmc::", "").split("(")[0]
    if "radix" in n or "canon" in n:
        acc[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for n, v in sorted(acc.items()):
    v = sorted(v)
    if v[-1] > 0.3: print("    %-40s %.3f ms med" % (n[:40], v[len(v) // 2]))
PY
  done
done
