// Decoding-side row kernel (inference path).
//
// lasr_logsoftmax_topk: one workgroup per row of logits [rows, V] (row stride ld,
// fp32 or bf16).  The row is staged once in LDS (coalesced 16-B-friendly reads over
// the vocab axis), then
//   logp[c]     = (x[c] - max) - log(sum_c exp(x[c] - max))     (torch's log_softmax form)
//   top-k       = k rounds of a block arg-max over the LDS row (descending value, ties
//                 to the smaller index), each winner masked to -inf for the next round
//   gathered[r] = logp[gather_idx[r]]  (optional; an index outside [0,V) yields -inf)
// It feeds CTC prefix beam search (u2.py:218-263: log_softmax then topk(beam) per
// frame) and attention rescoring (u2.py:300-313: log_softmax(h_attn) gathered at the
// hypothesis tokens).  HBM traffic = the logits once + k*(4+4) + 4 bytes per row.
#include "common.h"

namespace {

constexpr int kThreads = 256;

struct ArgMax {
  float v;
  int i;
};

LASR_DEV ArgMax better(ArgMax a, ArgMax b) {
  // larger value wins; equal values -> smaller index (NaN never produced: inputs finite
  // or -inf after masking)
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

LASR_DEV ArgMax wave_argmax(ArgMax a) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = better(a, b);
  }
  return a;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void logsoftmax_topk_kernel(
    const T* __restrict__ logits, int V, int64_t ld, int k, const int32_t* __restrict__ gidx,
    float* __restrict__ topv, int32_t* __restrict__ topi, float* __restrict__ gathered) {
  extern __shared__ float row[];  // V floats
  __shared__ float red[16];
  __shared__ float redv[16];
  __shared__ int redi[16];
  const int r = blockIdx.x;
  const T* x = logits + (int64_t)r * ld;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < V; c += kThreads) {
    float v = to_f(x[c]);
    row[c] = v;
    m = fmaxf(m, v);
  }
  m = block_max(m, red);
  float s = 0.f;
  for (int c = threadIdx.x; c < V; c += kThreads) s += __expf(row[c] - m);
  s = block_sum(s, red);
  const float lse = logf(s);
  if (gathered != nullptr && threadIdx.x == 0) {
    const int g = gidx[r];
    gathered[r] = (g >= 0 && g < V) ? (row[g] - m) - lse : -INFINITY;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int j = 0; j < k; ++j) {
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int c = threadIdx.x; c < V; c += kThreads) a = better(a, ArgMax{row[c], c});
    a = wave_argmax(a);
    __syncthreads();  // previous round's reads of row[] / redv[] are done
    if (lane == 0) {
      redv[w] = a.v;
      redi[w] = a.i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      ArgMax b{redv[0], redi[0]};
      for (int i = 1; i < kThreads / 64; ++i) b = better(b, ArgMax{redv[i], redi[i]});
      const int64_t o = (int64_t)r * k + j;
      topv[o] = (b.i < V) ? (b.v - m) - lse : -INFINITY;
      topi[o] = (b.i < V) ? b.i : -1;
      if (b.i < V) row[b.i] = -INFINITY;
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" int lasr_logsoftmax_topk(const void* logits, int dtype, int64_t rows, int V, int64_t ld,
                                    int k, const int32_t* gather_idx, float* topk_val,
                                    int32_t* topk_idx, float* gathered, void* stream) {
  if (rows <= 0) return LASR_OK;
  LASR_CHECK_ARG(V > 0 && V <= 16384, "logsoftmax_topk: V=%d outside [1, 16384]", V);
  LASR_CHECK_ARG(ld >= V, "logsoftmax_topk: ld=%lld < V=%d", (long long)ld, V);
  LASR_CHECK_ARG(k >= 0 && k <= V, "logsoftmax_topk: k=%d outside [0, V]", k);
  LASR_CHECK_ARG(k == 0 || (topk_val != nullptr && topk_idx != nullptr),
                 "logsoftmax_topk: k>0 needs topk outputs");
  LASR_CHECK_ARG((gather_idx == nullptr) == (gathered == nullptr),
                 "logsoftmax_topk: gather_idx and gathered go together");
  LASR_CHECK_ARG(rows <= 0x7fffffff, "logsoftmax_topk: too many rows");
  LASR_CHECK_ARG(dtype == LASR_F32 || dtype == LASR_BF16, "logsoftmax_topk: dtype %d", dtype);
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = (size_t)V * sizeof(float);
  if (dtype == LASR_F32)
    logsoftmax_topk_kernel<float><<<(int)rows, kThreads, lds, st>>>(
        (const float*)logits, V, ld, k, gather_idx, topk_val, topk_idx, gathered);
  else
    logsoftmax_topk_kernel<bf16_t><<<(int)rows, kThreads, lds, st>>>(
        (const bf16_t*)logits, V, ld, k, gather_idx, topk_val, topk_idx, gathered);
  return lasr_check_launch("logsoftmax_topk");
}
