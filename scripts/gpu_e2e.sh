# GPU: end-to-end (PCIe-inclusive) run of the C++ driver on a 10 Gbase synthetic FASTA
# file (SURVEY.md §8(d) layout, `kmc synth`): file -> device load (GPU parse vs host
# parse), step 1 (k=8 histogram), step 2 (distances), CSV.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
F=/tmp/kmc_e2e_$$.fa
trap 'rm -f $F' EXIT
R=${RECORDS:-10}; L=${LENGTH:-1000000000}
KMC=dna-kmeres-parallel_amd/bin/kmc
tm() { local t0=$(date +%s.%N); "$@"; local rc=$?; awk -v a=$t0 -v b=$(date +%s.%N) 'BEGIN{printf "wall %.2f s\n", b-a}' >> gpurun_out/e2e.log; return $rc; }
{ echo "nproc=$(nproc) cpu=$(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)"; df -h /tmp | tail -1; } > gpurun_out/e2e.log
tm timeout -k 10 300 $KMC synth $F $R $L >> gpurun_out/e2e.log 2>&1 || exit $?
ls -la $F >> gpurun_out/e2e.log
mkdir -p gpurun_out/e2e_gpu gpurun_out/e2e_host
for i in 1 2; do
  echo "== GPU parse, run $i" >> gpurun_out/e2e.log
  tm timeout -k 10 300 $KMC -k 8 --max-seqs 0 --out gpurun_out/e2e_gpu $F >> gpurun_out/e2e.log 2>&1 || exit $?
done
echo "== host parse" >> gpurun_out/e2e.log
tm timeout -k 10 300 $KMC -k 8 --max-seqs 0 --host-loader --out gpurun_out/e2e_host $F >> gpurun_out/e2e.log 2>&1 || exit $?
cmp gpurun_out/e2e_gpu/parallel_results.csv gpurun_out/e2e_host/parallel_results.csv && echo "CSV identical (GPU parse vs host parse)" >> gpurun_out/e2e.log
cat gpurun_out/e2e.log
