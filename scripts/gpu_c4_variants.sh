# GPU: C4 timing for the default build and every variant build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
: > gpurun_out/c4v.log
timeout -k 10 300 python scripts/cbench.py --configs c4 --iters 3 --cpu-sample-c4 0 | grep "^{" | sed 's/^/default /' >> gpurun_out/c4v.log || exit 1
for f in dna-kmeres-parallel_amd/lib/variants/*.so; do [ -e "$f" ] || continue
  KMC_LIB=$PWD/$f timeout -k 10 300 python scripts/cbench.py --configs c4 --iters 3 --cpu-sample-c4 0 | grep "^{" | sed "s|^|$(basename $f) |" >> gpurun_out/c4v.log || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/c4v.log'):
    n, j = l.split(' ', 1); d = json.loads(j); print('%-20s s_min %.4f s_med %.4f' % (n, d['s_min'], d['s_med']))"
