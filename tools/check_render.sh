#!/bin/bash
# The -m gpu suite, three interleaved C2 / C1 bench runs and a C2 rocprofv3 kernel-stats pass
# (output: gpurun_out/fi/).
set -o pipefail
mkdir -p gpurun_out/fi
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/fi/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/fi/pytest.log | tail -20; tail -3 gpurun_out/fi/pytest.log; exit 2; }
tail -1 gpurun_out/fi/pytest.log
for rep in 1 2 3; do
  for c in c2 c1; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-end-to-end > gpurun_out/fi/$c.$rep.log 2>&1 || { tail -5 gpurun_out/fi/$c.$rep.log; exit 3; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/fi/$c.$rep.log') if l.startswith('{')][-1]); print('$c', round(d['ms_per_step'],4))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fi/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/fi/prof.log 2>&1 || exit 4
head -8 gpurun_out/fi/prof/run_kernel_stats.csv | cut -d, -f1-4
