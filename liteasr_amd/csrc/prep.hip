// U2 integer bookkeeping on the device, bit-exact with the reference:
//   liteasr/models/u2.py:339-358 (_preprocess: ys_in, ys_mask), :323-333 (get_target),
//   :319-321 (get_pred_len), :146-148 (decoder mask = ys_mask | triangle_mask),
//   liteasr/utils/mask.py:8-27 (padding_mask), :30-90 (triangle_mask, stage = chunk),
//   liteasr/nets/transformer_encoder.py:117-120 (mask[:, :-2:2][:, :-2:2]: frame t' of
//   the subsampled sequence is padding iff 4*t' >= xlen).
#include "common.h"

LASR_DEV int64_t floordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

__global__ void u2_prep_kernel(const int64_t* xlens, const int64_t* ys, const int64_t* ylens,
                               int B, int L, int Tsub, int sos, int eos, int chunk,
                               int32_t* ys_in, int32_t* tgt, int32_t* tgt_ctc, uint8_t* dec_mask,
                               int dec_ld, uint8_t* enc_mask, int enc_ld, int32_t* pred_len,
                               int32_t* ylen32) {
  const int b = blockIdx.x;
  const int64_t xl = xlens[b];
  const int64_t yl = ylens[b];
  const int L1 = L + 1;
  if (threadIdx.x == 0) {
    pred_len[b] = (int32_t)floordiv(floordiv(xl - 1, 2) - 1, 2);
    ylen32[b] = (int32_t)yl;
    ys_in[(int64_t)b * L1] = sos;
  }
  for (int j = threadIdx.x; j < L; j += blockDim.x) {
    const int64_t y = ys[(int64_t)b * L + j];
    ys_in[(int64_t)b * L1 + 1 + j] = (int32_t)(y == -1 ? eos : y);
    tgt_ctc[(int64_t)b * L + j] = (int32_t)y;
  }
  for (int j = threadIdx.x; j < L1; j += blockDim.x) {
    int32_t v = (j < L) ? (int32_t)ys[(int64_t)b * L + j] : -1;
    if (j == yl) v = eos;
    tgt[(int64_t)b * L1 + j] = v;
  }
  // rows of dec_ld >= L1 bytes; the columns past L1 (row padding) are 1 = masked
  for (int e = threadIdx.x; e < L1 * dec_ld; e += blockDim.x) {
    const int i = e / dec_ld, j = e - i * dec_ld;
    dec_mask[(int64_t)b * L1 * dec_ld + e] = (uint8_t)((j >= L1) || (j >= yl + 1) || (j > i));
  }
  if (chunk <= 0) {
    for (int t = threadIdx.x; t < Tsub; t += blockDim.x)
      enc_mask[(int64_t)b * Tsub + t] = (uint8_t)((int64_t)4 * t >= xl);
  } else {
    for (int e = threadIdx.x; e < Tsub * enc_ld; e += blockDim.x) {
      const int i = e / enc_ld, j = e - i * enc_ld;
      enc_mask[(int64_t)b * Tsub * enc_ld + e] =
          (uint8_t)((j >= Tsub) || ((int64_t)4 * j >= xl) || ((j / chunk) > (i / chunk)));
    }
  }
}

extern "C" int lasr_u2_prep_ld(const int64_t* xlens, const int64_t* ys, const int64_t* ylens, int B,
                               int Tx, int L, int Tsub, int sos, int eos, int chunk, int32_t* ys_in,
                               int32_t* tgt, int32_t* tgt_ctc, uint8_t* dec_mask, int dec_ld,
                               uint8_t* enc_mask, int enc_ld, int32_t* pred_len, int32_t* ylen32,
                               void* stream) {
  (void)Tx;
  LASR_CHECK_ARG(dec_ld >= L + 1 && (chunk <= 0 || enc_ld >= Tsub), "lasr_u2_prep: mask row stride too small");
  if (B <= 0) return LASR_OK;
  u2_prep_kernel<<<B, 256, 0, (hipStream_t)stream>>>(xlens, ys, ylens, B, L, Tsub, sos, eos, chunk,
                                                     ys_in, tgt, tgt_ctc, dec_mask, dec_ld, enc_mask,
                                                     chunk > 0 ? enc_ld : Tsub, pred_len, ylen32);
  return lasr_check_launch("u2_prep");
}

extern "C" int lasr_u2_prep(const int64_t* xlens, const int64_t* ys, const int64_t* ylens, int B,
                            int Tx, int L, int Tsub, int sos, int eos, int chunk, int32_t* ys_in,
                            int32_t* tgt, int32_t* tgt_ctc, uint8_t* dec_mask, uint8_t* enc_mask,
                            int32_t* pred_len, int32_t* ylen32, void* stream) {
  return lasr_u2_prep_ld(xlens, ys, ylens, B, Tx, L, Tsub, sos, eos, chunk, ys_in, tgt, tgt_ctc, dec_mask,
                         L + 1, enc_mask, Tsub, pred_len, ylen32, stream);
}
