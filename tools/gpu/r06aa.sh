# round 6 A/B (experiment): non-temporal Y stores in the column-block launches (1: all blocks, 2: partials only)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06aa
mkdir -p $O
cd $R
for v in 0 1 2 0 1 2; do
  SRG_BLOCK_NT=$v timeout -k 10 300 python -u bench.py --config products --steps 10 --warmup 3 --pmc off --no-cpu-baseline > $O/products_nt$v.json 2> $O/products_nt$v.err || exit 1
  python -c "import json; r=json.load(open('$O/products_nt$v.json')); print('products block_nt $v', round(r['ms_per_step']/10, 4), r['parity_vs_oracle']['bit_exact'])" >> $O/summary.txt
done
