cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/calib && rm -rf gpurun_out/calib/*
run() { timeout -k 10 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run 300 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B --output-format csv -d gpurun_out/calib/a -o c -- python3 scripts/pmc_calib.py > gpurun_out/calib/a.log 2>&1
run 300 rocprofv3 --pmc TCC_BUBBLE TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_RDREQ_DRAM --output-format csv -d gpurun_out/calib/b -o c -- python3 scripts/pmc_calib.py > gpurun_out/calib/b.log 2>&1
run 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/c -o c -- python3 scripts/pmc_calib.py > gpurun_out/calib/c.log 2>&1
run 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/d -o c -- python3 scripts/pmc_calib.py > gpurun_out/calib/d.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/calib > gpurun_out/calib/summary.txt
cat gpurun_out/calib/summary.txt
