# GPU: K4 phase split (scripts/c4_prof.py) for every -DKMC_CANON_PROF variant build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for f in dna-kmeres-parallel_amd/lib/variants/*prof*.so; do
  echo "== $(basename $f)"
  KMC_LIB=$PWD/$f timeout -k 10 300 python3 scripts/c4_prof.py 2>&1 | grep -E "iter|probe" || exit 1
done
