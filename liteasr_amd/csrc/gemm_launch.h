// The bf16 launch table of lasr_gemm (gemm.hip): tile / ring-depth selection over the
// template instances of gemm_kernel.h.  Instantiated per operand layout in gemm_l{0..3}.hip
// so the instance-heavy translation units compile in parallel.
#pragma once
#include "gemm_kernel.h"

template <bool AKC, bool BKC, typename TC>
void launch_bf16(const GemmP& p, int BM, int BN, int ks, int nw, bool glds, dim3 grid, hipStream_t st) {
  (void)nw;  // no 8-wave generic instance is planned (gemm.hip gemm_plan)
  if (glds && ks == 2 && BM < 256) {
    // 64-deep ring stages (two 32-deep sub-tiles per wait + barrier); shallower rings keep
    // the LDS footprint at the KS = 1 instances' occupancy where it fits
    if (BN == 256) gemm_bf16_glds_kernel<128, 256, AKC, BKC, TC, 2, 1, G_LIN, 2><<<grid, 256, 0, st>>>(p);
    else if (BM == 128 && BN == 128) gemm_bf16_glds_kernel<128, 128, AKC, BKC, TC, 2, 2, G_LIN, 2><<<grid, 256, 0, st>>>(p);
    else if (BM == 128) gemm_bf16_glds_kernel<128, 64, AKC, BKC, TC, 3, 2, G_LIN, 2><<<grid, 256, 0, st>>>(p);
    else if (BN == 128) gemm_bf16_glds_kernel<64, 128, AKC, BKC, TC, 3, 2, G_LIN, 2><<<grid, 256, 0, st>>>(p);
    else {
      // the 64 x 64 launches of the N = d family: input gradients (B N-contiguous, bf16 out) and
      // the residual projections (fp32 out)
      const int e = epi_code(p);
#define L64(E) gemm_bf16_glds_kernel<64, 64, AKC, BKC, TC, 3, 3, G_LIN, 2, 4, E><<<grid, 256, 0, st>>>(p)
      if constexpr (AKC && std::is_same<TC, bf16_t>::value) {
        if (e == EPI_PLAIN) { L64(EPI_PLAIN); return; }
      }
      if constexpr (AKC && !BKC && std::is_same<TC, bf16_t>::value) {
        if (e == EPI_AUX_GATE) { L64(EPI_AUX_GATE); return; }  // the decoder's FFN dz
      }
      if constexpr (AKC && BKC && std::is_same<TC, bf16_t>::value) {
        if (e == EPI_RELU_GATE_DROP) { L64(EPI_RELU_GATE_DROP); return; }  // the decoder's FFN fc1
      }
#undef L64
      if constexpr (AKC && BKC && std::is_same<TC, float>::value) {
        if (e == EPI_RES_DROP) {
          gemm_bf16_glds_kernel<64, 64, AKC, BKC, TC, 3, 3, G_LIN, 2, 4, EPI_RES_DROP><<<grid, 256, 0, st>>>(p);
          return;
        }
      }
      gemm_bf16_glds_kernel<64, 64, AKC, BKC, TC, 3, 3, G_LIN, 2><<<grid, 256, 0, st>>>(p);
    }
    return;
  }
  if (glds) {
    if (BM == 256 && BN == 256) gemm_bf16_glds_kernel<256, 256, AKC, BKC, TC, 3, 1><<<grid, 256, 0, st>>>(p);
    else if (BM == 256) gemm_bf16_glds_kernel<256, 128, AKC, BKC, TC, 3, 2><<<grid, 256, 0, st>>>(p);
    else if (BN == 256) {
      // the FFN fc1 forward (A, B K-contiguous) and its dz GEMM (B N-contiguous), bf16 out
      const int e = epi_code(p);
      if constexpr (AKC && BKC && std::is_same<TC, bf16_t>::value) {
        if (e == EPI_SWISH_GATE_DROP) {
          gemm_bf16_glds_kernel<128, 256, AKC, BKC, TC, 3, 2, G_LIN, 1, 4, EPI_SWISH_GATE_DROP><<<grid, 256, 0, st>>>(p);
          return;
        }
      }
      if constexpr (AKC && !BKC && std::is_same<TC, bf16_t>::value) {
        if (e == EPI_AUX_GATE) {
          gemm_bf16_glds_kernel<128, 256, AKC, BKC, TC, 3, 2, G_LIN, 1, 4, EPI_AUX_GATE><<<grid, 256, 0, st>>>(p);
          return;
        }
        if (e == EPI_AUX_RELU) {  // the subsampling output projection's input gradient
          gemm_bf16_glds_kernel<128, 256, AKC, BKC, TC, 3, 2, G_LIN, 1, 4, EPI_AUX_RELU><<<grid, 256, 0, st>>>(p);
          return;
        }
      }
      gemm_bf16_glds_kernel<128, 256, AKC, BKC, TC, 3, 2><<<grid, 256, 0, st>>>(p);
    }
    else if (BM == 128 && BN == 128) {
      // (the CTC head and the decoder memory K/V projections: bias only)
      if constexpr (AKC && BKC && std::is_same<TC, bf16_t>::value) {
        if (epi_code(p) == EPI_PLAIN) {
          gemm_bf16_glds_kernel<128, 128, AKC, BKC, TC, 3, 3, G_LIN, 1, 4, EPI_PLAIN><<<grid, 256, 0, st>>>(p);
          return;
        }
      }
      gemm_bf16_glds_kernel<128, 128, AKC, BKC, TC, 3><<<grid, 256, 0, st>>>(p);
    }
    else if (BM == 128) {
      // (the q/k/v projection: bias only)
      if constexpr (AKC && BKC && std::is_same<TC, bf16_t>::value) {
        if (epi_code(p) == EPI_PLAIN) {
          gemm_bf16_glds_kernel<128, 64, AKC, BKC, TC, 4, 3, G_LIN, 1, 4, EPI_PLAIN><<<grid, 256, 0, st>>>(p);
          return;
        }
      }
      gemm_bf16_glds_kernel<128, 64, AKC, BKC, TC, 4><<<grid, 256, 0, st>>>(p);
    }
    else if (BN == 128) {
      // (the batched attention GEMMs of the materialised path: alpha / plain)
      if constexpr (AKC && std::is_same<TC, bf16_t>::value) {
        if (epi_code(p) == EPI_PLAIN) {
          gemm_bf16_glds_kernel<64, 128, AKC, BKC, TC, 4, 3, G_LIN, 1, 4, EPI_PLAIN><<<grid, 256, 0, st>>>(p);
          return;
        }
      }
      gemm_bf16_glds_kernel<64, 128, AKC, BKC, TC, 4><<<grid, 256, 0, st>>>(p);
    }
    else gemm_bf16_glds_kernel<64, 64, AKC, BKC, TC, 4><<<grid, 256, 0, st>>>(p);
    return;
  }
  if (BM == 128 && BN == 128) gemm_bf16_kernel<128, 128, AKC, BKC, TC><<<grid, 256, 0, st>>>(p);
  else if (BM == 128) gemm_bf16_kernel<128, 64, AKC, BKC, TC><<<grid, 256, 0, st>>>(p);
  else if (BN == 128) gemm_bf16_kernel<64, 128, AKC, BKC, TC><<<grid, 256, 0, st>>>(p);
  else gemm_bf16_kernel<64, 64, AKC, BKC, TC><<<grid, 256, 0, st>>>(p);
}

