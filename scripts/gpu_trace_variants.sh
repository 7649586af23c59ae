# GPU: per-kernel times (rocprofv3 --kernel-trace --stats of scripts/kbench.py) for the
# default build and every diagnostic variant in lib/variants, k = $KS.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/vtrace && rm -rf gpurun_out/vtrace/*
for f in "" dna-kmeres-parallel_amd/lib/variants/*.so; do
  name=$(basename "${f:-libkmc.so}" .so)
  if [ -n "$f" ]; then export KMC_LIB=$PWD/$f; else unset KMC_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vtrace/$name -o kt -- \
    python3 scripts/kbench.py --ks ${KS:-9,13} --iters ${ITERS:-2} > gpurun_out/vtrace/$name.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/vtrace/$name.log; exit 1; }
  echo "== $name"
  python3 - gpurun_out/vtrace/$name <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "synth" in n or "rocclr" in n:
        continue
    print("  %-70s %4s %9.3f ms" % (n.replace("kmc::(anonymous namespace)::", "")[:70], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
