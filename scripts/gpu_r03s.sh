# GPU (round 3): reduce slots from the shard geometry (no slot_rec listing): dense
# parity tests + fuzz, then per-rank steps same-box against r03p (slots listed from slot_rec).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03s && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
run 600 python -u -m pytest tests/test_dense_gpu.py tests/test_cli.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run 600 python -u scripts/fuzz_dense.py --cases 30 --seed 45 > $O/fuzz.log 2>&1
tail -1 $O/fuzz.log
for r in 1 2; do
  run 300 python scripts/shardbench.py --worlds 1,2,8 > $O/shard_new$r.log 2>&1
  KMC_LIB=$V/libkmc_r03p.so run 300 python scripts/shardbench.py --worlds 1,2,8 > $O/shard_old$r.log 2>&1
  echo "== new $r"; grep '^{' $O/shard_new$r.log | cut -c1-150
  echo "== old $r"; grep '^{' $O/shard_old$r.log | cut -c1-150
done
