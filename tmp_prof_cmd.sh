export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01prof
mkdir -p $O
timeout -k 10 300 python3 $R/tools/sweep.py --nt > $O/sweep.json 2> $O/sweep.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 $R/bench.py --steps 3 --no-cpu-baseline > $O/trace_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o fetch --output-format csv -- python3 $R/tools/spmm_probe.py > $O/probe.json 2> $O/pmc_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o write --output-format csv -- python3 $R/tools/spmm_probe.py > $O/probe2.json 2> $O/pmc_write.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/cal_fetch -o calf --output-format csv -- python3 $R/tools/spmm_probe.py --identity > $O/cal_probe.json 2> $O/cal_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/cal_write -o calw --output-format csv -- python3 $R/tools/spmm_probe.py --identity > $O/cal_probe2.json 2> $O/cal_write.err
echo "rc=$?"
