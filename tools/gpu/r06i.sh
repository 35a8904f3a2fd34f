# round 6: fp64 blocked steps -- parity after the W=256 hub windows, then the products sweep over
# column blocks, whole-hub thresholds and block-launch occupancy (SRG_CHEBY64_WAVES: an experiment knob of
# that build, removed after the sweep -- profiles/r06i_cheby64_plan_sweep.txt)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06i
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_wavelet_gpu.py > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/probes/cheby64_parts_probe.py products --plan > $O/plan_w0.json 2> $O/plan_w0.err &&
SRG_CHEBY64_WAVES=6 timeout -k 10 300 python -u tools/probes/cheby64_parts_probe.py products --plan > $O/plan_w6.json 2> $O/plan_w6.err &&
SRG_CHEBY64_WAVES=4 timeout -k 10 300 python -u tools/probes/cheby64_parts_probe.py products --plan > $O/plan_w4.json 2> $O/plan_w4.err
