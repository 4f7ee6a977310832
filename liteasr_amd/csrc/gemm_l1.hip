// lasr_gemm bf16 launch table, A K-contiguous x B N-contiguous instances (gemm_launch.h).
#include "gemm_launch.h"

template void launch_bf16<true, false, float>(const GemmP&, int, int, int, int, bool, dim3, hipStream_t);
template void launch_bf16<true, false, bf16_t>(const GemmP&, int, int, int, int, bool, dim3, hipStream_t);
