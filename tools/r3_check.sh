#!/bin/bash
# Round-3 iteration check on the GPU box: targeted GPU tests, then the C5 / ViT / C2 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r3}
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread ${TESTS:-tests/test_vit.py tests/test_seg.py} -m gpu > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 7; }
tail -1 gpurun_out/${T}_pytest.log
for cfg in ${CFGS:-c5 vit c2}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end > gpurun_out/${T}_bench_$cfg.log 2>&1 || { tail -20 gpurun_out/${T}_bench_$cfg.log; exit 8; }
  python - "$cfg" "gpurun_out/${T}_bench_$cfg.log" <<'PY'
import json, sys
cfg, f = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(f) if l.startswith("{")][-1])
r = d.get("roofline", {})
if cfg == "vit":
    print(cfg, {k: round(v["ms_per_pass"], 3) for k, v in d["models"].items()})
else:
    print(cfg, round(d["ms_per_step"], 3), "ms", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items() if k.endswith("_ms") or k in ("frac", "achieved")})
PY
done
