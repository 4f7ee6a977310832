// lasr_gemm bf16 launch table, A M-contiguous x B N-contiguous instances (gemm_launch.h).
#include "gemm_launch.h"

template void launch_bf16<false, false, float>(const GemmP&, int, int, int, int, bool, dim3, hipStream_t);
template void launch_bf16<false, false, bf16_t>(const GemmP&, int, int, int, int, bool, dim3, hipStream_t);
