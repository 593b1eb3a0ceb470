set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/tmr
for e in 1 4 1 4; do
  SCENEDINO_AMD_TIMER_EVERY=$e timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/tmr/c2_$e.log 2>&1 || exit 2
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/tmr/c2_$e.log') if l.startswith('{')][0]); print('c2 every $e', d['ms_per_step'], d['roofline']['kernel_ms'] if 'kernel_ms' in d['roofline'] else d['roofline'].get('achieved'))"
done
for e in 1 4; do
  SCENEDINO_AMD_TIMER_EVERY=$e timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > gpurun_out/tmr/c5_$e.log 2>&1 || exit 3
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/tmr/c5_$e.log') if l.startswith('{')][0]); print('c5 every $e', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
