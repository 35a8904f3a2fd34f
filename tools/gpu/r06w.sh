# round 6 A/B: the fp32 hub fork's dispatch delay (10 us default vs none vs 5), arxiv and products
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06w
mkdir -p $O
cd $R
for v in 10 0 5 10 0; do
  SRG_HUB_DELAY_US=$v timeout -k 10 300 python -u bench.py --config arxiv --steps 40 --warmup 5 --pmc off --no-cpu-baseline > $O/arxiv_d$v.json 2> $O/arxiv_d$v.err || exit 1
  python -c "import json; r=json.load(open('$O/arxiv_d$v.json')); print('arxiv delay $v', round(r['ms_per_step']/5, 4), r['parity_vs_oracle']['bit_exact'])" >> $O/summary.txt
done
for v in 10 0 10 0; do
  SRG_HUB_DELAY_US=$v timeout -k 10 300 python -u bench.py --config products --steps 10 --warmup 3 --pmc off --no-cpu-baseline > $O/products_d$v.json 2> $O/products_d$v.err || exit 1
  python -c "import json; r=json.load(open('$O/products_d$v.json')); print('products delay $v', round(r['ms_per_step']/10, 4), r['parity_vs_oracle']['bit_exact'])" >> $O/summary.txt
done
