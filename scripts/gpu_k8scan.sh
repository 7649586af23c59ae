# GPU: same-box A/B of the k = 8 scan interval (lib/variants), alternating order,
# kernel time from scripts/kbench.py (HIP events, median of 20 after warm-up).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/k8scan && mkdir -p $O && rm -rf $O/*
for r in 1 2 3; do
  for v in ${VARS:-s64 s128 s256 s0}; do
    KMC_LIB=$PWD/dna-kmeres-parallel_amd/lib/variants/libkmc_$v.so timeout -k 10 120 python3 scripts/kbench.py --ks 8 --iters 20 --tag $v >> $O/kb.log 2>&1 || { tail -5 $O/kb.log; exit 1; }
  done
done
grep '^{' $O/kb.log | python3 -c "import sys,json; [print('%-6s %.4f ms' % (d['lib'], d['ms_med'])) for d in map(json.loads, sys.stdin)]"
