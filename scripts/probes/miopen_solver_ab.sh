set -o pipefail
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/mi_$name.log 2>&1 || { echo "$name failed"; exit 1; }; echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/mi_$name.log | head -1)"; }
run base A=1
run nowrw MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
run nobwd MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
run noboth MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
