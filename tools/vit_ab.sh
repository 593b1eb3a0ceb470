#!/bin/bash
# Diagnostic: ViT encoder bench under the runtime switches (LN fusion, register-streaming
# small GEMM, 4- vs 8-wave attention), one line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python bench.py --config vit --steps 20 --warmup 5 > gpurun_out/vitab.log 2>&1 || { tail -5 gpurun_out/vitab.log; exit 7; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/vitab.log') if l.startswith('{')][-1]); print('$*', {k: round(v['ms_per_pass'],3) for k,v in d['models'].items()})"
}
run X=all_new
run SCENEDINO_AMD_LN_GEMM=0
run SD_GEMM_DIR=0
run SD_ATTN=dir4
run SCENEDINO_AMD_LN_GEMM=0 SD_GEMM_DIR=0 SD_ATTN=dir4
