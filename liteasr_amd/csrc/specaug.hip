// SpecAugment on the padded feature batch in HBM.
//
// Reference: liteasr/utils/transform/spec_augment.py:14-125, run per utterance on the CPU in
// DataLoader workers (liteasr/dataset/asr_dataset.py:118).  Here the host draws every random
// number in the reference's order (liteasr_amd/utils/transform/spec_augment.py) and packs
// them into a per-utterance int32 plan; two launches then apply the whole batch:
//
//   specaug_warp_kernel  time warp (:18-48).  Rows [0, warped) are the Pillow BICUBIC
//                        resize of rows [0, center), rows [warped, xlen) that of rows
//                        [center, xlen); rows >= xlen (padding) are copied.  Pillow's float
//                        ('F' image) vertical pass is reproduced operation for operation in
//                        double precision with contraction off, so the result is
//                        bit-identical to Image.resize (checked against Pillow 12.2).
//   specaug_mask_kernel  freq masks (:50-79) then time masks (:81-114), in draw order, one
//                        workgroup per utterance: each mask fills its [lo, hi) range with
//                        0 or with the mean of the utterance's current xlen x F values
//                        (double sums, fixed reduction trees -> deterministic; the sum is
//                        updated by each fill instead of being recomputed).
//
// Plan row (stride P >= 4 + 2 * (nf + nt) int32):
//   [0] center  [1] warped (0 = no warp)  [2] nf  [3] nt  then nf freq [lo, hi) pairs and
//   nt time [lo, hi) pairs, already clipped to [0, F] / [0, xlen].
//
// Both kernels are HBM-bound byte movers: the warp reads x once and writes out once
// (8 B per element); the mean fill rereads the warped utterance once (4 B per element,
// L2-hot) plus the masked regions.
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int SA_ROWS = 16;      // output rows per warp-kernel workgroup
constexpr int SA_THREADS = 256;
constexpr int SA_TPR = SA_THREADS / SA_ROWS;  // tap threads per row
constexpr int SA_KMAX = 32;      // taps kept in LDS per row
constexpr int SM_THREADS = 1024;

// Resample.c bicubic_filter (a = -0.5), evaluated in the same operation order.
LASR_DEV double bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// One output pixel of Pillow's vertical BICUBIC resize nin -> nout rows
// (precompute_coeffs + ImagingResampleVertical_32bpc): src points at column c of row 0
// of the segment, ld is the row stride in floats.
LASR_DEV float resize_px(const float* __restrict__ src, int64_t ld, int nin, int nout, int yy) {
  const double scale = (double)(float)nin / nout;
  const double fscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * fscale;
  const double center = 0.0 + (yy + 0.5) * scale;
  const double ss = 1.0 / fscale;
  int lo = (int)(center - support + 0.5);
  if (lo < 0) lo = 0;
  int hi = (int)(center + support + 0.5);
  if (hi > nin) hi = nin;
  const int n = hi - lo;
  double ww = 0.0;
  for (int x = 0; x < n; ++x) ww += bicubic((x + lo - center + 0.5) * ss);
  double acc = 0.0;
  for (int x = 0; x < n; ++x) {
    double k = bicubic((x + lo - center + 0.5) * ss);
    if (ww != 0.0) k /= ww;
    acc += (double)src[(int64_t)(x + lo) * ld] * k;
  }
  return (float)acc;
}

// Each workgroup produces SA_ROWS output rows.  The bicubic taps of a row are shared by its
// F pixels, so they are computed once into LDS (weights by one thread per tap, the
// normalising sum by one thread per row in Pillow's sequential order, then w / ww per tap)
// and every pixel thread accumulates over them in tap order.  Rows with more than SA_KMAX
// taps (a segment shrunk by more than ~8x) fall back to per-pixel evaluation.
__global__ void __launch_bounds__(SA_THREADS)
specaug_warp_kernel(const float* __restrict__ x, float* __restrict__ out,
                    const int64_t* __restrict__ xlens, const int32_t* __restrict__ plan, int P,
                    int Tmax, int F, double* __restrict__ part) {
  __shared__ double kw[SA_ROWS][SA_KMAX];
  __shared__ int rlo[SA_ROWS], rn[SA_ROWS];  // first tap (segment-relative), tap count
  // rn: -1 = copy row (source row in rlo, absolute), -2 = per-pixel fallback
  const int b = blockIdx.y;
  const int r0 = blockIdx.x * SA_ROWS;
  const int t = (int)min(max(xlens[b], (int64_t)0), (int64_t)Tmax);
  const int center = plan[(int64_t)b * P + 0];
  int warped = plan[(int64_t)b * P + 1];
  if (center <= 0 || center >= t || warped <= 0 || warped >= t) warped = 0;  // malformed: copy
  const float* xb = x + (int64_t)b * Tmax * F;
  float* ob = out + (int64_t)b * Tmax * F;
  const int nrow = min(SA_ROWS, Tmax - r0);
  const int tid = threadIdx.x;
  // phase 1: per-row tap range; per-tap raw weights
  {
    const int i = tid / SA_TPR, x0 = tid % SA_TPR;
    const int r = r0 + i;
    if (i < nrow) {
      int lo = 0, n = -1;
      if (warped == 0 || r >= t) {
        lo = r;
      } else {
        const int nin = r < warped ? center : t - center;
        const int nout = r < warped ? warped : t - warped;
        const int yy = r < warped ? r : r - warped;
        if (nin == nout) {
          lo = (r < warped ? 0 : center) + yy;
        } else {
          const double scale = (double)(float)nin / nout;
          const double fscale = scale < 1.0 ? 1.0 : scale;
          const double support = 2.0 * fscale;
          const double c = 0.0 + (yy + 0.5) * scale;
          const double ss = 1.0 / fscale;
          lo = (int)(c - support + 0.5);
          if (lo < 0) lo = 0;
          int hi = (int)(c + support + 0.5);
          if (hi > nin) hi = nin;
          n = hi - lo;
          if (n > SA_KMAX) {
            n = -2;
          } else {
            for (int xx = x0; xx < n; xx += SA_TPR) kw[i][xx] = bicubic((xx + lo - c + 0.5) * ss);
          }
        }
      }
      if (x0 == 0) {
        rlo[i] = lo;
        rn[i] = n;
      }
    }
  }
  __syncthreads();
  // phase 2: normalising sum in tap order (one thread per row), then w / ww per tap
  __shared__ double rww[SA_ROWS];
  if (tid < nrow) {
    double ww = 0.0;
    for (int xx = 0; xx < rn[tid]; ++xx) ww += kw[tid][xx];
    rww[tid] = ww;
  }
  __syncthreads();
  {
    const int i = tid / SA_TPR, x0 = tid % SA_TPR;
    if (i < nrow && rww[i] != 0.0)
      for (int xx = x0; xx < rn[i]; xx += SA_TPR) kw[i][xx] = kw[i][xx] / rww[i];
  }
  __syncthreads();
  // phase 3: pixels (+ this block's share of the utterance sum for the mean fill)
  double psum = 0.0;
  for (int e = tid; e < nrow * F; e += SA_THREADS) {
    const int i = e / F, c = e - i * F;
    const int r = r0 + i;
    const int n = rn[i];
    float v;
    if (n == -1) {
      v = xb[(int64_t)rlo[i] * F + c];
    } else {
      const int in0 = r < warped ? 0 : center;
      const float* src = xb + (int64_t)in0 * F + c;
      if (n == -2) {
        const int nin = r < warped ? center : t - center;
        const int nout = r < warped ? warped : t - warped;
        v = resize_px(src, F, nin, nout, r < warped ? r : r - warped);
      } else {
        const float* s = src + (int64_t)rlo[i] * F;
        double acc = 0.0;
        for (int xx = 0; xx < n; ++xx) acc += (double)s[(int64_t)xx * F] * kw[i][xx];
        v = (float)acc;
      }
    }
    ob[(int64_t)r * F + c] = v;
    if (r < t) psum += (double)v;
  }
  if (part != nullptr) {
    __shared__ double red[SA_THREADS / 64];
    for (int o = 32; o > 0; o >>= 1) psum += __shfl_xor(psum, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = psum;
    __syncthreads();
    if (tid == 0) {
      double s = 0.0;
      for (int i = 0; i < SA_THREADS / 64; ++i) s += red[i];
      part[(int64_t)b * gridDim.x + blockIdx.x] = s;
    }
  }
}

LASR_DEV double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < SM_THREADS / 64; ++i) s += red[i];
    red[SM_THREADS / 64] = s;
  }
  __syncthreads();
  s = red[SM_THREADS / 64];
  __syncthreads();
  return s;
}

// Mean fill without rereading the utterance: the warp kernel leaves one partial sum per
// (utterance, row block); the mask kernel adds them in a fixed tree, then for each mask
// subtracts the sum of the region it overwrites and adds fill * count, so every mask sees
// the mean of the utterance as left by the previous one (reference :77-78, :112-113).
__global__ void __launch_bounds__(SM_THREADS)
specaug_mask_kernel(float* __restrict__ out, const int64_t* __restrict__ xlens,
                    const int32_t* __restrict__ plan, int P, int Tmax, int F, int zero,
                    const double* __restrict__ part, int npart) {
  __shared__ double red[SM_THREADS / 64 + 1];
  const int b = blockIdx.x;
  const int t = (int)min(max(xlens[b], (int64_t)0), (int64_t)Tmax);
  const int32_t* pl = plan + (int64_t)b * P;
  const int nf = max(pl[2], 0), nt = max(pl[3], 0);
  if (nf + nt == 0 || 4 + 2 * (nf + nt) > P) return;  // nothing to do / malformed plan row
  float* ob = out + (int64_t)b * Tmax * F;
  const double n = (double)t * F;
  double s = 0.0;
  if (!zero) {
    for (int i = threadIdx.x; i < npart; i += SM_THREADS) s += part[(int64_t)b * npart + i];
    s = block_sum(s, red);
  }
  const int last = nf + nt - 1;
  for (int m = 0; m <= last; ++m) {
    const int ext = m < nf ? F : t;  // ranges are clipped on the host; re-clip defensively
    const int lo = max(pl[4 + 2 * m], 0), hi = min(pl[5 + 2 * m], ext);
    if (hi <= lo) continue;
    const float fill = zero ? 0.f : (float)(s / n);
    const bool track = !zero && m < last;  // later masks need the updated sum
    // freq mask: columns [lo, hi) of rows [0, t); time mask: rows [lo, hi), all columns.
    // Either way a (rows x w) box: thread -> (column, first row), stride rpi rows.
    const int w = m < nf ? hi - lo : F;
    const int r_begin = m < nf ? 0 : lo, r_end = m < nf ? t : hi;
    const int c0 = m < nf ? lo : 0;
    const int rpi = SM_THREADS / w;  // w <= F; F <= SM_THREADS checked on the host
    const int j = threadIdx.x / w, c = c0 + threadIdx.x - j * w;
    const bool act = j < rpi;
    if (track) {
      double rs = 0.0;
      if (act) {
        int r = r_begin + j;
        for (; r + 3 * rpi < r_end; r += 4 * rpi) {  // 4 loads in flight, summed in row order
          const float v0 = ob[(int64_t)r * F + c], v1 = ob[(int64_t)(r + rpi) * F + c];
          const float v2 = ob[(int64_t)(r + 2 * rpi) * F + c], v3 = ob[(int64_t)(r + 3 * rpi) * F + c];
          rs += (double)v0;
          rs += (double)v1;
          rs += (double)v2;
          rs += (double)v3;
        }
        for (; r < r_end; r += rpi) rs += (double)ob[(int64_t)r * F + c];
      }
      rs = block_sum(rs, red);  // all region reads complete before any fill below
      s = s - rs + (double)fill * ((double)(r_end - r_begin) * w);
    }
    if (act)
      for (int r = r_begin + j; r < r_end; r += rpi) ob[(int64_t)r * F + c] = fill;
    __syncthreads();
  }
}

}  // namespace

extern "C" int64_t lasr_spec_augment_ws_bytes(int B, int Tmax) {
  return (int64_t)(B > 0 ? B : 0) * cdiv(Tmax > 0 ? Tmax : 0, SA_ROWS) * (int64_t)sizeof(double);
}

extern "C" int lasr_spec_augment(const float* x, float* out, const int64_t* xlens,
                                 const int32_t* plan, int plan_stride, int B, int Tmax, int F,
                                 int replace_with_zero, void* ws, int64_t ws_bytes,
                                 void* stream) {
  LASR_CHECK_ARG(B >= 0 && Tmax >= 0 && F > 0 && F <= SM_THREADS,
                 "spec_augment: bad shape B=%d T=%d F=%d (F <= %d)", B, Tmax, F, SM_THREADS);
  LASR_CHECK_ARG(plan_stride >= 4, "spec_augment: plan stride %d < 4", plan_stride);
  LASR_CHECK_ARG(x != out, "spec_augment: out must not alias x");
  const int64_t need = lasr_spec_augment_ws_bytes(B, Tmax);
  LASR_CHECK_ARG(replace_with_zero || (ws != nullptr && ws_bytes >= need),
                 "spec_augment: workspace %lld bytes < %lld", (long long)ws_bytes,
                 (long long)need);
  if (B == 0 || Tmax == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  const int nblk = (int)cdiv(Tmax, SA_ROWS);
  double* part = replace_with_zero ? nullptr : (double*)ws;
  specaug_warp_kernel<<<dim3((unsigned)nblk, (unsigned)B), SA_THREADS, 0, st>>>(
      x, out, xlens, plan, plan_stride, Tmax, F, part);
  int rc = lasr_check_launch("spec_augment_warp");
  if (rc != LASR_OK) return rc;
  specaug_mask_kernel<<<B, SM_THREADS, 0, st>>>(out, xlens, plan, plan_stride, Tmax, F,
                                                replace_with_zero, part, nblk);
  return lasr_check_launch("spec_augment_mask");
}
