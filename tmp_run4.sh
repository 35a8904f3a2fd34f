export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01c
mkdir -p $O
timeout -k 10 900 python -m pytest $R/tests -m gpu -q > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $O/pytest_gpu.log
timeout -k 10 300 python3 $R/tools/sweep.py --thresholds 32 --n 400000 --n-edges 63000000 > $O/sweep_mall.json 2> $O/sweep_mall.err &&
timeout -k 10 300 python3 $R/tools/sweep.py --thresholds 32 --n 9000000 --n-edges 63000000 > $O/sweep_big.json 2> $O/sweep_big.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o f --output-format csv -- python3 $R/tools/spmm_probe.py > $O/probe.json 2> $O/pf.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o w --output-format csv -- python3 $R/tools/spmm_probe.py > /dev/null 2> $O/pw.err &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/ph -o h --output-format csv -- python3 $R/tools/spmm_probe.py > /dev/null 2> $O/ph.err &&
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $O/pd -o d --output-format csv -- python3 $R/tools/spmm_probe.py > /dev/null 2> $O/pd.err
echo "all rc=$?"
