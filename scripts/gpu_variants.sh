# GPU box: time measurement variants (scripts/build_variant.py) against each other,
# alternating, in separate processes: bash scripts/gpu_variants.sh TAG PASSES "ARGS" V1 V2 ...
# ARGS: a python script and its arguments ("scripts/kbench.py --ks 8"); Vi: lib/variants/libkmc_Vi.so, or "product".
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=$1; PASSES=$2; ARGS=$3; shift 3
O=gpurun_out/$TAG && mkdir -p $O
for p in $(seq $PASSES); do
    for v in "$@"; do
        if [ "$v" = product ]; then L=dna-kmeres-parallel_amd/lib/libkmc.so; else L=dna-kmeres-parallel_amd/lib/variants/libkmc_$v.so; fi
        KMC_LIB=$L timeout -k 10 300 python $ARGS >> $O/variants.log 2>&1
        rc=$?; if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 $O/variants.log; exit $rc; fi
        echo "pass $p $v done"
    done
done
grep '^{' $O/variants.log
