# GPU: refresh the round's bench evidence: rocprofv3 trace + HBM PMC of the bench
# command (scripts/profile_bench.sh), the default bench line, and the SQ/LDS PMC
# groups of the k=8 kernel (scripts/gpu_pmc.sh).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
bash scripts/profile_bench.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
grep "^{" gpurun_out/bench.log
KS=8 bash scripts/gpu_pmc.sh > gpurun_out/pmc_k8.txt 2>&1 || { tail -5 gpurun_out/pmc_k8.txt; exit 1; }
head -60 gpurun_out/pmc_k8.txt
