# round 6 A/B (experiment): block 0's whole rows on a second stream beside the column blocks
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06z
mkdir -p $O
cd $R
for v in 0 1 0 1; do
  SRG_WHOLE_CONC=$v timeout -k 10 300 python -u bench.py --config products --steps 10 --warmup 3 --pmc off --no-cpu-baseline > $O/products_c$v.json 2> $O/products_c$v.err || exit 1
  python -c "import json; r=json.load(open('$O/products_c$v.json')); print('products conc $v', round(r['ms_per_step']/10, 4), r['roofline']['kernel_ms'], r['parity_vs_oracle']['bit_exact'])" >> $O/summary.txt
done
for v in 0 1; do
  SRG_WHOLE_CONC=$v timeout -k 10 300 python -u bench.py --config products --aggregate weighted --steps 5 --warmup 2 --pmc off --no-cpu-baseline > $O/agg_c$v.json 2> $O/agg_c$v.err || exit 1
  python -c "import json; r=json.load(open('$O/agg_c$v.json')); print('aggregate conc $v', round(r['ms_per_step'], 3), (r.get('parity_vs_oracle') or {}).get('bit_exact'))" >> $O/summary.txt
done
SRG_WHOLE_CONC=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_plan_gpu.py tests/test_aggregate_gpu.py tests/test_plan_lifecycle_gpu.py > $O/pytest_conc.log 2>&1
tail -1 $O/pytest_conc.log >> $O/summary.txt
