# GPU (round 3): per-call kernel breakdown of C3R with the sampled partition.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03h && mkdir -p $O && rm -rf $O/*
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/c3r -o t -- python3 scripts/cbench.py --configs c3r --iters 2 > $O/c3r.log 2>&1 || { tail -5 $O/c3r.log; exit 1; }
grep '^{' $O/c3r.log | cut -c1-150
python3 scripts/trace_calls.py $O/c3r place 2
