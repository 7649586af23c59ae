# GPU: C4 under a kernel + memory-copy trace; the timeline of the last call
# (scripts/timeline.py) shows where the time between the canon_* kernels goes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/c4tl && mkdir -p $O && rm -rf $O/*
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t -o t -- python3 scripts/cbench.py --configs ${CONFIGS:-c4} --iters 2 --cpu-sample-c4 0 --cpu-sample-c3 0 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
grep '^{' $O/run.log | cut -c1-300
python3 scripts/timeline.py $O/t ${TL_FROM:-canon_count_kernel} > $O/timeline.txt && cat $O/timeline.txt
