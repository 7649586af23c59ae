cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash scripts/gpu_radix3.sh || exit 1
O=gpurun_out/r4d && mkdir -p $O && rm -rf $O/*
for grp in WRITE_SIZE "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  n=$(echo $grp | cut -c1-5)
  KMC_LIB=$PWD/dna-kmeres-parallel_amd/lib/variants/libkmc_r4direct.so timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $O/$n -o run -- python3 scripts/kbench.py --ks 13 --iters 2 > $O/$n.log 2>&1 || { echo "pmc failed"; exit 1; }
done
python3 scripts/pmc_summary.py $O | grep -A4 "hist_kernel\|place"
