# GPU (round 4): K3b segments of 16 entries (a whole 128-byte line, a lane quad storing two 16-byte
# pieces per lane) -- new -- against 8 (seg8, the shipped 64-byte segments); C4 and C4R via cbench under
# the kernel trace, same box, two alternating rounds; then the GPU tests.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04al && mkdir -p $O && rm -rf $O/*
run() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
V=$PWD/dna-kmeres-parallel_amd/lib/variants
for r in 1 2; do
  for v in ${C4V:-seg8 new}; do
    L=$V/libkmc_$v.so; [ $v = new ] && L=$PWD/dna-kmeres-parallel_amd/lib/libkmc.so
    KMC_LIB=$L run 400 rocprofv3 --kernel-trace --output-format csv -d $O/$v$r -o t -- python3 scripts/cbench.py --configs ${CB:-c4,c4r} --iters 3 --cpu-sample-c4 0 > $O/$v$r.log 2>&1
    echo "== $v $r $(grep -o '"s_med": [0-9.]*' $O/$v$r.log | tr '\n' ' ')"; python3 scripts/trace_split.py $O/$v$r | grep -E "fine|sort|table"
  done
done
run 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_hash_gpu.py tests/test_dense_gpu.py > $O/tests_hash.log 2>&1 || { tail -30 $O/tests_hash.log; exit 1; }
tail -1 $O/tests_hash.log
run 600 python3 scripts/fuzz_canonical.py > $O/fuzz_canonical.log 2>&1 || { tail -20 $O/fuzz_canonical.log; exit 1; }
tail -1 $O/fuzz_canonical.log
