#!/bin/bash
# k_project iteration: projection parity tests, then k_project's time in C2 and C5 profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/proj
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_pack_proj.py tests/test_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread -k "proj or channels_last or end_to_end" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 3; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 4; }
python3 - <<'PY'
import csv, glob
for c in ("c2", "c5"):
    f = glob.glob(f"gpurun_out/proj/{c}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "k_project" in r["Name"] or "k_render_tile" in r["Name"]:
            print(c, r["Name"][:40], r["Calls"], r["AverageNs"])
PY
