cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/encprof
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/encprof/s16 -o run -- \
  python bench.py --config encode --models vit-s16 --steps 5 --warmup 3 > gpurun_out/encprof/s16.log 2>&1 || exit 7
f=$(find gpurun_out/encprof/s16 -name '*kernel_trace.csv' | head -1)
python tools/trace_pass.py $f k_patchify --list > gpurun_out/encprof/pass_s16.txt 2>&1
