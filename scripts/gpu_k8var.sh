# GPU: k = 8 kernel time (kbench, 10 Gbase) for the default build and every
# diagnostic build in lib/variants/, interleaved twice to see box drift.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/k8var && mkdir -p $O && : > $O/kb.jsonl
for rep in 1 2; do
  timeout -k 10 120 python3 scripts/kbench.py --ks 8 --iters 20 >> $O/kb.jsonl 2>/dev/null || exit 1
  for f in dna-kmeres-parallel_amd/lib/variants/*.so; do
    KMC_LIB=$PWD/$f timeout -k 10 120 python3 scripts/kbench.py --ks 8 --iters 20 >> $O/kb.jsonl 2>/dev/null || exit 1
  done
done
cat $O/kb.jsonl
