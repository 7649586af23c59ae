# GPU: canonical parity tests, C4 + C4R (default build, parity-checked) under a kernel
# trace, then C4 for the diagnostic builds in lib/variants/ (no checks); per-call
# canon_* kernel times (scripts/c4_calls.py).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
CONFIGS=c4,c4r VAR_SKIP=1 bash scripts/gpu_c4_trace.sh > gpurun_out/c4ab.log 2>&1 || { tail -30 gpurun_out/c4ab.log; exit 1; }
grep passed gpurun_out/c4t/tests.log; grep "^default" gpurun_out/c4ab.log
python3 scripts/c4_calls.py gpurun_out/c4t/default | sed -n '2p;$p'
mkdir -p gpurun_out/c4v && rm -rf gpurun_out/c4v/*
for f in dna-kmeres-parallel_amd/lib/variants/*.so; do [ -e "$f" ] || continue; v=$(basename $f .so)
  KMC_LIB=$PWD/$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4v/$v -o t -- python3 scripts/cbench.py --configs ${VCFGS:-c4} --iters 2 --no-check --cpu-sample-c4 0 --cpu-sample-c3 0 > gpurun_out/c4v/$v.log 2>&1 || { tail -5 gpurun_out/c4v/$v.log; exit 1; }
  echo "== $v"; python3 scripts/c4_calls.py gpurun_out/c4v/$v | sed -n "2p;\$p"
done
