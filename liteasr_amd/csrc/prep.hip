// U2 integer bookkeeping on the device, bit-exact with the reference:
//   liteasr/models/u2.py:339-358 (_preprocess: ys_in, ys_mask), :323-333 (get_target),
//   :319-321 (get_pred_len), :146-148 (decoder mask = ys_mask | triangle_mask),
//   liteasr/utils/mask.py:8-27 (padding_mask), :30-90 (triangle_mask, stage = chunk),
//   liteasr/nets/transformer_encoder.py:117-120 (mask[:, :-2:2][:, :-2:2]: frame t' of
//   the subsampled sequence is padding iff 4*t' >= xlen).
//
// One launch writes every output, the streaming chunk mask included (config 4):
// blockIdx.y == 0 does utterance b's bookkeeping, blockIdx.y >= 1 a run of 16 chunk-mask rows.
// A chunk-mask row i is a threshold: key j is masked iff j >= min(T', ceil(xlen/4),
// (i div c + 1) c), so each thread writes whole 16-B vectors.  The chunk size c is a launch
// argument (fixed), a device scalar (a captured graph replays whatever the host wrote there),
// or drawn on the device per step from (seed, the step counter) -- the dynamic-chunk
// training mode, replayable inside a graph.
#include "common.h"

LASR_DEV int64_t floordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

enum { CH_NONE = 0, CH_FIXED = 1, CH_DEVICE = 2, CH_SAMPLE = 3 };
constexpr int PREP_ROWS = 16;  // chunk-mask rows per block (16 threads per row, 16 B each)

// The dynamic chunk draw (WeNet's add_optional_chunk_mask distribution over T' frames):
// r uniform in [1, T'-1] from the step's hash; r > T'/2 -> full context (c = T'), else
// c = r mod cmax + 1.  Mirrored in liteasr_amd/models/_fused.py (dynamic_chunk_size).
LASR_DEV int chunk_draw(uint64_t seed, uint64_t ctr, int Tsub, int cmax) {
  if (Tsub <= 1) return Tsub > 0 ? Tsub : 1;
  const uint64_t s = seed + ctr * 0xD1B54A32D192ED03ull;
  const uint32_t key = mix32((uint32_t)s ^ mix32((uint32_t)(s >> 32) + 0x9E3779B9u));
  const uint32_t h = mix32(key ^ 0x5BD1E995u);
  const int r = 1 + (int)(h % (uint32_t)(Tsub - 1));
  return r > Tsub / 2 ? Tsub : r % cmax + 1;
}

__global__ void u2_prep_kernel(const int64_t* xlens, const int64_t* ys, const int64_t* ylens,
                               int B, int L, int Tsub, int sos, int eos, int mode, int chunk,
                               int32_t* chunk_dev, const uint64_t* ctr, uint64_t seed, int cmax,
                               int32_t* ys_in, int32_t* tgt, int32_t* tgt_ctc, uint8_t* dec_mask,
                               int dec_ld, uint8_t* key_mask, uint8_t* chunk_mask, int chunk_ld,
                               int32_t* pred_len, int32_t* ylen32) {
  const int b = blockIdx.x;
  const int64_t xl = xlens[b];
  if (blockIdx.y > 0) {  // chunk-mask rows
    int c = chunk;
    if (mode == CH_DEVICE) c = chunk_dev[0];
    else if (mode == CH_SAMPLE) c = chunk_draw(seed, ctr[0], Tsub, cmax);
    if (c <= 0 || c > Tsub) c = Tsub;  // full context
    const int64_t klim = xl <= 0 ? 0 : floordiv(xl + 3, 4);  // first j with 4 j >= xlen
    const bool vec = chunk_ld % 16 == 0 && ((uintptr_t)chunk_mask & 15) == 0;
    const int nv = chunk_ld / 16;
    const int i = (blockIdx.y - 1) * PREP_ROWS + threadIdx.x / 16;
    if (i >= Tsub) return;
    const int64_t lim = min(min((int64_t)Tsub, klim), (int64_t)(i / c + 1) * c);
    uint8_t* rowp = chunk_mask + ((int64_t)b * Tsub + i) * chunk_ld;
    if (!vec) {  // rows that are not 16-B vectors (the unpadded lasr_u2_prep layout)
      for (int j = threadIdx.x % 16; j < chunk_ld; j += 16) rowp[j] = (uint8_t)((int64_t)j >= lim);
      return;
    }
    uint4* row = reinterpret_cast<uint4*>(rowp);
    for (int v = threadIdx.x % 16; v < nv; v += 16) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) x |= (uint32_t)((int64_t)(16 * v + 4 * q + k) >= lim) << (8 * k);
        w[q] = x;
      }
      row[v] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return;
  }
  const int64_t yl = ylens[b];
  const int L1 = L + 1;
  if (threadIdx.x == 0) {
    pred_len[b] = (int32_t)floordiv(floordiv(xl - 1, 2) - 1, 2);
    ylen32[b] = (int32_t)yl;
    ys_in[(int64_t)b * L1] = sos;
    if (b == 0 && mode == CH_SAMPLE && chunk_dev) chunk_dev[0] = chunk_draw(seed, ctr[0], Tsub, cmax);
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
  if (key_mask)
    for (int t = threadIdx.x; t < Tsub; t += blockDim.x)
      key_mask[(int64_t)b * Tsub + t] = (uint8_t)((int64_t)4 * t >= xl);
}

extern "C" int lasr_u2_prep_chunk(const int64_t* xlens, const int64_t* ys, const int64_t* ylens, int B,
                                  int L, int Tsub, int sos, int eos, int chunk_mode, int chunk,
                                  int32_t* chunk_dev, const uint64_t* ctr, uint64_t chunk_seed, int chunk_max,
                                  int32_t* ys_in, int32_t* tgt, int32_t* tgt_ctc, uint8_t* dec_mask, int dec_ld,
                                  uint8_t* key_mask, uint8_t* chunk_mask, int chunk_ld, int32_t* pred_len,
                                  int32_t* ylen32, void* stream) {
  LASR_CHECK_ARG(chunk_mode >= CH_NONE && chunk_mode <= CH_SAMPLE, "lasr_u2_prep_chunk: bad chunk_mode");
  LASR_CHECK_ARG(dec_ld >= L + 1, "lasr_u2_prep: decoder mask row stride too small");
  LASR_CHECK_ARG(Tsub >= 0 && L >= 0, "lasr_u2_prep: negative size");
  if (chunk_mode != CH_NONE) {
    LASR_CHECK_ARG(chunk_mask && chunk_ld >= Tsub, "lasr_u2_prep_chunk: chunk mask needs rows of >= T' bytes");
    LASR_CHECK_ARG(chunk_mode != CH_FIXED || chunk > 0, "lasr_u2_prep_chunk: fixed chunk must be > 0");
    LASR_CHECK_ARG(chunk_mode != CH_DEVICE || chunk_dev, "lasr_u2_prep_chunk: device chunk needs chunk_dev");
    LASR_CHECK_ARG(chunk_mode != CH_SAMPLE || (ctr && chunk_max > 0), "lasr_u2_prep_chunk: sampled chunk needs the step counter and chunk_max > 0");
  }
  if (B <= 0) return LASR_OK;
  const int ry = chunk_mode == CH_NONE ? 0 : (Tsub + PREP_ROWS - 1) / PREP_ROWS;
  u2_prep_kernel<<<dim3(B, 1 + ry), 256, 0, (hipStream_t)stream>>>(
      xlens, ys, ylens, B, L, Tsub, sos, eos, chunk_mode, chunk, chunk_dev, ctr, chunk_seed, chunk_max,
      ys_in, tgt, tgt_ctc, dec_mask, dec_ld, key_mask, chunk_mask, chunk_ld, pred_len, ylen32);
  return lasr_check_launch("u2_prep");
}

extern "C" int lasr_u2_prep_ld(const int64_t* xlens, const int64_t* ys, const int64_t* ylens, int B,
                               int Tx, int L, int Tsub, int sos, int eos, int chunk, int32_t* ys_in,
                               int32_t* tgt, int32_t* tgt_ctc, uint8_t* dec_mask, int dec_ld,
                               uint8_t* enc_mask, int enc_ld, int32_t* pred_len, int32_t* ylen32,
                               void* stream) {
  (void)Tx;
  LASR_CHECK_ARG(chunk <= 0 || enc_ld >= Tsub, "lasr_u2_prep: mask row stride too small");
  if (chunk > 0)
    return lasr_u2_prep_chunk(xlens, ys, ylens, B, L, Tsub, sos, eos, CH_FIXED, chunk, nullptr, nullptr, 0, 0,
                              ys_in, tgt, tgt_ctc, dec_mask, dec_ld, nullptr, enc_mask, enc_ld, pred_len,
                              ylen32, stream);
  return lasr_u2_prep_chunk(xlens, ys, ylens, B, L, Tsub, sos, eos, CH_NONE, 0, nullptr, nullptr, 0, 0, ys_in,
                            tgt, tgt_ctc, dec_mask, dec_ld, enc_mask, nullptr, 0, pred_len, ylen32, stream);
}

extern "C" int lasr_u2_prep(const int64_t* xlens, const int64_t* ys, const int64_t* ylens, int B,
                            int Tx, int L, int Tsub, int sos, int eos, int chunk, int32_t* ys_in,
                            int32_t* tgt, int32_t* tgt_ctc, uint8_t* dec_mask, uint8_t* enc_mask,
                            int32_t* pred_len, int32_t* ylen32, void* stream) {
  return lasr_u2_prep_ld(xlens, ys, ylens, B, Tx, L, Tsub, sos, eos, chunk, ys_in, tgt, tgt_ctc, dec_mask,
                         L + 1, enc_mask, Tsub, pred_len, ylen32, stream);
}
