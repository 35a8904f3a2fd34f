#!/bin/bash
# GPU-box script: calibration of the 2 x FETCH_SIZE + WRITE_SIZE traffic formula on GATHERS -- the
# hop kernel on a random permutation operator at the products size (every X row gathered once as a
# random whole-row read, no reuse: known bytes) at d = 128 and 256, beside the identity operator
# (a sequential read).  -> gpurun_out/<tag>/pmc_gather_calibration.txt
# Usage: pmc_calib.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
bash "$R/tools/gpu/pmc_probe.sh" "$T" perm_d128 --config products --permutation --d 128 --reps 3 > /dev/null &&
bash "$R/tools/gpu/pmc_probe.sh" "$T" perm_d256 --config products --permutation --d 256 --reps 3 > /dev/null &&
bash "$R/tools/gpu/pmc_probe.sh" "$T" ident_d128 --identity --d 128 --reps 3 > /dev/null &&
python3 - "$O" > "$O/pmc_gather_calibration.txt" <<'PY'
import json, os, sys
o = sys.argv[1]
print("operator                      d   pmc read GB  known read GB  ratio   pmc write GB  known write GB  ratio   L2 hit")
for name in ("perm_d128", "perm_d256", "ident_d128"):
    rec = json.load(open(os.path.join(o, f"pmc_{name}.json")))
    probe = json.load(open(os.path.join(o, name, "probe.json")))
    n, d = probe["n"], probe["d"]
    # X rows (4d B), column id + value (8 B), schedule slot (4 B) per row; int64 row pointers
    known_r = n * 4 * d + n * 12 + (n + 1) * 8
    known_w = n * 4 * d
    r, w = rec["hbm_read_bytes_per_launch"], rec["hbm_write_bytes_per_launch"]
    print(f"{probe['config']:28s} {d:4d}  {r / 1e9:10.3f}  {known_r / 1e9:12.3f}  {r / known_r:6.3f}  "
          f"{w / 1e9:11.3f}  {known_w / 1e9:13.3f}  {w / known_w:6.3f}  {rec.get('l2_hit_rate', float('nan')):.3f}")
print("read = 2 x FETCH_SIZE, write = WRITE_SIZE (bench.py's traffic formula), per launch, median of 3 reps")
PY
