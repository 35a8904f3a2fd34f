# round 6: fp32 hop with more whole hub rows (probe)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06l
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/probes/whole_hub_f32_probe.py products > $O/whole_hub_f32.json 2> $O/whole_hub_f32.err
