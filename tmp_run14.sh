export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01m
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 $R/bench.py --steps 3 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o f --output-format csv -- python3 $R/tools/spmm_probe.py > $O/probe.json 2> $O/pf.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o w --output-format csv -- python3 $R/tools/spmm_probe.py > /dev/null 2> $O/pw.err &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/ph -o h --output-format csv -- python3 $R/tools/spmm_probe.py > /dev/null 2> $O/ph.err
echo "all rc=$?"
