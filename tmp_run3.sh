export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01b
mkdir -p $O
timeout -k 10 900 python -m pytest $R/tests -m gpu -q -x > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
rocprofv3 -L > $O/counters.txt 2>&1;
timeout -k 10 300 python3 $R/tools/sweep.py --nt --thresholds 0,8,16,32,64,128 > $O/sweep.json 2> $O/sweep.err &&
for T in 0 -1; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$T -o f --output-format csv -- python3 $R/tools/spmm_probe.py --heavy-threshold $T > $O/probe_$T.json 2> $O/pf_$T.err &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw_$T -o w --output-format csv -- python3 $R/tools/spmm_probe.py --heavy-threshold $T > /dev/null 2> $O/pw_$T.err &&
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/cf_$T -o cf --output-format csv -- python3 $R/tools/spmm_probe.py --identity --heavy-threshold $T > $O/cal_$T.json 2> $O/cf_$T.err &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/cw_$T -o cw --output-format csv -- python3 $R/tools/spmm_probe.py --identity --heavy-threshold $T > /dev/null 2> $O/cw_$T.err &&
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/ph_$T -o h --output-format csv -- python3 $R/tools/spmm_probe.py --heavy-threshold $T > /dev/null 2> $O/ph_$T.err || break
done
echo "all rc=$?"
