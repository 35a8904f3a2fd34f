# round 6: the any-order hub launch (SRG_HUB_ANY_ORDER=1 variant) against the default library on arxiv;
# parity of the variant; its kernel timeline
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06e
mkdir -p $O
cd $R
bash tools/gpu/lib_ab_quick.sh r06e 3 "--config arxiv --steps 20 --warmup 5" scalable-roubust-gnn_amd/lib/variants/libsrgnn_hip_base.so scalable-roubust-gnn_amd/lib/variants/libsrgnn_hip_anyorder.so &&
SRGNN_HIP_LIB=$R/scalable-roubust-gnn_amd/lib/variants/libsrgnn_hip_anyorder.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_full_size_gpu.py -k "not rmat26 and not papers100M and not int64 and not products" > $O/pytest_anyorder.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
SRGNN_HIP_LIB=$R/scalable-roubust-gnn_amd/lib/variants/libsrgnn_hip_anyorder.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ta -o ta --output-format csv -- python3 $R/bench.py --config arxiv --steps 10 --warmup 3 --no-cpu-baseline --pmc off > $O/trace_arxiv.json 2> $O/trace_arxiv.err &&
python3 $R/tools/trace_timeline.py $O/ta --last 24 > $O/arxiv_timeline_anyorder.txt
