cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/diag && mkdir -p $O && rm -rf $O/*
timeout -k 10 300 python scripts/diag_dense.py 1.0 > $O/diag.log 2>&1; rc=$?; cat $O/diag.log | tail -20; exit $rc
