# GPU box: time measurement variants (scripts/build_variant.py) against each other,
# alternating, in separate processes: bash scripts/gpu_variants.sh TAG PASSES "ARGS" V1 V2 ...
# ARGS: a python script and its arguments ("scripts/kbench.py --ks 8"); Vi: lib/variants/libkmc_Vi.so, or "product".
# PROF=1: each run under rocprofv3 --kernel-trace --stats, with its per-kernel averages printed.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=$1; PASSES=$2; ARGS=$3; shift 3
O=gpurun_out/$TAG && mkdir -p $O
for p in $(seq $PASSES); do
    for v in "$@"; do
        if [ "$v" = product ]; then L=dna-kmeres-parallel_amd/lib/libkmc.so; else L=dna-kmeres-parallel_amd/lib/variants/libkmc_$v.so; fi
        if [ -n "$PROF" ]; then
            KMC_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${p}_$v -o v \
                -- python3 $ARGS >> $O/variants.log 2>&1
        else
            KMC_LIB=$L timeout -k 10 300 python $ARGS >> $O/variants.log 2>&1
        fi
        rc=$?; if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 $O/variants.log; exit $rc; fi
        echo "pass $p $v done"
        if [ -n "$PROF" ]; then
            python3 - $O/prof_${p}_$v $v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]
print(sys.argv[2], "; ".join("%s %s x %.3f ms" % (r["Name"].split("(")[0].replace("kmc::(anonymous namespace)::", "")[:40], r["Calls"], float(r["AverageNs"]) / 1e6) for r in rows))
PY
        fi
    done
done
grep '^{\|median' $O/variants.log
