# GPU: canonical GPU tests, the direct-output probe, and a same-box A/B of the
# canonical output path (direct vs pk + place copy) on C4 / C4R under the kernel
# trace.  usage: bash scripts/gpu_ab_canon.sh TAG [ROUNDS]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=${1:-ab}; O=gpurun_out/$TAG; mkdir -p $O
bash scripts/gpu_run.sh $TAG "tests:hash or canonical or abi" || exit $?
run() { local lim=$1 log=$2; shift 2; timeout -k 10 $lim "$@" > $log 2>&1; local rc=$?; echo "[$log] rc=$rc"; grep -v amdgpu.ids $log | grep '^{\|call\|share\|queued' | cut -c1-300; if [ $rc -ne 0 ]; then tail -20 $log; exit $rc; fi; }
run 400 $O/probe.log python scripts/canon_direct_probe.py
for i in $(seq 1 ${2:-2}); do
run 600 $O/ab_direct_$i.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_d$i -o cb -- python3 scripts/cbench.py --configs c4,c4r --iters 3 --cpu-sample-c4 0 --canon-direct 1
run 600 $O/ab_pk_$i.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p$i -o cb -- python3 scripts/cbench.py --configs c4,c4r --iters 3 --cpu-sample-c4 0 --canon-direct 0
done
