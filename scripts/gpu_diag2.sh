cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/diag && mkdir -p $O && rm -rf $O/*
for v in flat restart; do echo $v; KMC_LIB=$PWD/dna-kmeres-parallel_amd/lib/variants/libkmc_$v.so timeout -k 10 300 python scripts/diag_dense.py 1.0 > $O/diag_$v.log 2>&1 || exit 1; tail -6 $O/diag_$v.log | cut -c1-110; done
