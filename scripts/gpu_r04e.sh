# GPU (round 4): the integer VALU issue costs (scripts/valu_microbench.hip), then the
# templated canonical walks (K1 / K3a by orientation and key width, branch-free K1
# adds) against the previous build (lib/variants/libkmc_k3base.so: the same source
# before the change) on C4, same box, alternating; then the canonical + full-size
# tests and the validation profiles of scripts/gpu_r04c.sh on the new build.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04e && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 120 scripts/bin/valu_microbench > $O/valu.txt 2>&1
cat $O/valu.txt
V=$PWD/dna-kmeres-parallel_amd/lib/variants
for r in 1 2; do
  for v in k3base new; do
    L=$V/libkmc_$v.so; [ $v = new ] && L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/cbench.py --configs ${CBAB:-c4} --iters 3 --cpu-sample-c4 0 > $O/$v$r.log 2>&1
    echo "== $v $r $(grep -o '"s_med": [0-9.]*' $O/$v$r.log | tr '\n' ' ')"; python3 scripts/trace_kernels.py $O/$v$r canon_
  done
done
[ -n "$NOVALID" ] && exit 0
TFILES="tests/test_hash_gpu.py tests/test_baseline_configs_gpu.py" TESTS="not zzz" PMC3=1 SHARD=1 bash scripts/gpu_r04c.sh
