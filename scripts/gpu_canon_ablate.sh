cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r05u && mkdir -p $O
for p in 1 2; do for v in product nowb norsv nowbrsv; do
  if [ $v = product ]; then L=dna-kmeres-parallel_amd/lib/libkmc.so; else L=dna-kmeres-parallel_amd/lib/variants/libkmc_$v.so; fi
  KMC_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p${p}_$v -o cb -- python3 scripts/canon_time.py --configs c4,c4r --iters 3 > $O/p${p}_$v.log 2>&1 || { echo "fail $v"; tail -5 $O/p${p}_$v.log; exit 1; }
  grep median $O/p${p}_$v.log
done; done
