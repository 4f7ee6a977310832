// Launch of the grouped split-K weight-gradient kernel (gemm_kernel.h gemm_dw_group_kernel);
// the entry point lasr_gemm_dw_group (gemm.hip) plans and validates the problems.
#include "gemm_kernel.h"

int launch_dw_group(const DwGroupP& g, int BM, int BN, int blocks, hipStream_t st) {
  if (BM == 64 && BN == 64) gemm_dw_group_kernel<64, 64, 3, 3><<<blocks, 256, 0, st>>>(g);
  else if (BM == 64 && BN == 128) gemm_dw_group_kernel<64, 128, 3, 2><<<blocks, 256, 0, st>>>(g);
  else if (BM == 128 && BN == 64) gemm_dw_group_kernel<128, 64, 3, 2><<<blocks, 256, 0, st>>>(g);
  else if (BM == 128 && BN == 128) gemm_dw_group_kernel<128, 128, 2, 2><<<blocks, 256, 0, st>>>(g);
  // 8 waves (512 threads), one workgroup per CU
  else if (BM == 256 && BN == 128) gemm_dw_group_kernel<256, 128, 3, 1, 8><<<blocks, 512, 0, st>>>(g);
  else return -1;
  return 0;
}
