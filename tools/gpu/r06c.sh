# round 6: kernel-trace timelines of the arxiv and products hops (hub fork / chain / main launches)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ta -o ta --output-format csv -- python3 $R/bench.py --config arxiv --steps 10 --warmup 3 --no-cpu-baseline --pmc off > $O/arxiv.json 2> $O/arxiv.err &&
python3 $R/tools/trace_timeline.py $O/ta --last 40 > $O/arxiv_timeline.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tp -o tp --output-format csv -- python3 $R/bench.py --config products --steps 3 --warmup 2 --no-cpu-baseline --pmc off > $O/products.json 2> $O/products.err &&
python3 $R/tools/trace_timeline.py $O/tp --last 60 > $O/products_timeline.txt
