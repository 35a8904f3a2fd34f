# round 6: fp64 hub workgroups for the Chebyshev step -- parity, then the products probe
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_wavelet_gpu.py tests/test_capi.py > $O/pytest_wavelet.log 2>&1 &&
timeout -k 10 300 python -u tools/probes/cheby64_parts_probe.py products --hub-only > $O/cheby64_hub.json 2> $O/cheby64_hub.err
