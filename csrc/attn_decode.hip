// Single-query attention against a KV cache (autoregressive decode), gfx950.
//
// Replaces the reference's generation path (generate.py:37-42), which re-runs the full model
// over the whole context for every new token (no KV cache; Llama3.py:131-155 materialises the
// [B,H,T,T] scores each time).  Here K/V of past positions live in a cache laid out
// [B, G, Tmax, hd] (one contiguous 2*hd-byte row per key, GQA-native: the H/G query heads of a
// kv group read the same rows), and each new token costs one pass over the cache.
//
// One workgroup per (batch, query head), 256 threads:
//   1. scores: every thread owns keys k = tid, tid+256, ...; it streams its key's row (16-B
//      loads) and dots it with q held in registers (fp32);  scores -> LDS;
//   2. softmax: block max / sum over the scores (exp2 with folded log2e);
//   3. out[d] = sum_k p_k V[k][d]: thread = (d-chunk of 8, key phase), rows read coalesced,
//      partial sums combined through LDS in a fixed order.
// Memory-bound (reads each cached row once per query head); fp32 accumulation throughout.
#include "api.h"

namespace bllm {

BLLM_DEBUG_WORD(attn_decode)

constexpr int DEC_THREADS = 256;
constexpr int DEC_MAXL = 8192;  // LDS score buffer (32 KiB)

// APPEND (graph-replayed decode, the position known only on the device): q, the new key and
// the new value come from the packed qkv row of the token (row stride qs); L = *pos + 1 and key
// L - 1 is read from that row, while the first query head of each kv group also writes it into
// the caches at row *pos (no block of this launch reads cache row *pos, so no ordering needed).
template <typename T, int HD, bool APPEND>
__global__ __launch_bounds__(DEC_THREADS) void attn_decode_k(const T* __restrict__ q, T* __restrict__ kc,
                                                             T* __restrict__ vc, T* __restrict__ out,
                                                             int H, int G, int Tmax, int L, float scale,
                                                             const int* __restrict__ pos, long qs) {
  constexpr int VEC = 8;               // elements per 16-B load
  constexpr int NC = HD / VEC;         // 16-B chunks per row
  constexpr int KPH = DEC_THREADS / NC;  // key phases in the output pass
  __shared__ float sc[DEC_MAXL];
  __shared__ float red[DEC_THREADS / 64];
  __shared__ float part[KPH][HD];
  const int bh = blockIdx.x, h = bh % H, b = bh / H;
  const int g = h / (H / G);
  const int tid = threadIdx.x;
  const T* qr = APPEND ? q + (long)b * qs + (long)h * HD : q + ((long)b * H + h) * HD;
  T* kb = kc + ((long)b * G + g) * (long)Tmax * HD;
  T* vb = vc + ((long)b * G + g) * (long)Tmax * HD;
  const T* knew = nullptr;
  const T* vnew = nullptr;
  if constexpr (APPEND) {
    int p = *pos;
    BLLM_DASSERT(p >= 0 && p < Tmax && p < DEC_MAXL, DBG_DECODE_POS);
#ifdef BLLM_KERNEL_DEBUG
    p = p < 0 ? 0 : (p >= Tmax ? Tmax - 1 : p);
    p = p >= DEC_MAXL ? DEC_MAXL - 1 : p;
#endif
    L = p + 1;
    knew = q + (long)b * qs + (long)(H + g) * HD;
    vnew = q + (long)b * qs + (long)(H + G + g) * HD;
    if (h % (H / G) == 0 && tid < 2 * (HD / 8)) {  // one block per kv group appends k and v
      const int c = tid % (HD / 8);
      if (tid < HD / 8) st16(kb + (long)p * HD + c * 8, ld16(knew + c * 8));
      else st16(vb + (long)p * HD + c * 8, ld16(vnew + c * 8));
    }
  }
  const float c = scale * 1.4426950408889634f;

  float qf[HD];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const Vec16<T> v = ld16(qr + i * VEC);
#pragma unroll
    for (int j = 0; j < VEC; ++j) qf[i * VEC + j] = to_f(v.v[j]);
  }
  // 1. scores (log2 domain)
  float mx = -INFINITY;
  for (int k = tid; k < L; k += DEC_THREADS) {
    const T* kr = (APPEND && k == L - 1) ? knew : kb + (long)k * HD;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const Vec16<T> v = ld16(kr + i * VEC);
#pragma unroll
      for (int j = 0; j < VEC; ++j) s += qf[i * VEC + j] * to_f(v.v[j]);
    }
    s *= c;
    sc[k] = s;
    mx = fmaxf(mx, s);
  }
  // 2. softmax statistics
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = red[0];
#pragma unroll
  for (int i = 1; i < DEC_THREADS / 64; ++i) mx = fmaxf(mx, red[i]);
  __syncthreads();
  float sum = 0.f;
  for (int k = tid; k < L; k += DEC_THREADS) {
    const float p = exp2f(sc[k] - mx);
    sc[k] = p;
    sum += p;
  }
  sum = wave_sum(sum);
  if ((tid & 63) == 0) red[tid >> 6] = sum;
  __syncthreads();
  sum = 0.f;
#pragma unroll
  for (int i = 0; i < DEC_THREADS / 64; ++i) sum += red[i];
  const float inv = 1.f / sum;
  // 3. weighted V sum: thread = (chunk ci, key phase kp)
  const int ci = tid % NC, kp = tid / NC;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  for (int k = kp; k < L; k += KPH) {
    const Vec16<T> v = ld16(((APPEND && k == L - 1) ? vnew : vb + (long)k * HD) + ci * VEC);
    const float p = sc[k];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] += p * to_f(v.v[j]);
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) part[kp][ci * VEC + j] = acc[j];
  __syncthreads();
  for (int d = tid; d < HD; d += DEC_THREADS) {
    float o = 0.f;
#pragma unroll
    for (int p2 = 0; p2 < KPH; ++p2) o += part[p2][d];
    out[((long)b * H + h) * HD + d] = from_f<T>(o * inv);
  }
}

int attn_decode_max_len() { return DEC_MAXL; }

void attn_decode(DType dt, const void* q, const void* kc, const void* vc, void* out, int B, int H, int G, int hd,
                 int Tmax, int L, hipStream_t s) {
  const float scale = 1.f / sqrtf((float)hd);
  dim3 grid(B * H), block(DEC_THREADS);
#define L_(TT, HDD) hipLaunchKernelGGL((attn_decode_k<TT, HDD, false>), grid, block, 0, s, (const TT*)q, (TT*)kc, \
                                       (TT*)vc, (TT*)out, H, G, Tmax, L, scale, nullptr, 0L)
  if (dt == DType::BF16) {
    if (hd == 128) L_(bf16_t, 128); else L_(bf16_t, 64);
  } else {
    if (hd == 128) L_(f16_t, 128); else L_(f16_t, 64);
  }
#undef L_
}

void attn_decode_append(DType dt, const void* qkv, void* kc, void* vc, void* out, const int* pos, int B, int H,
                        int G, int hd, int Tmax, hipStream_t s) {
  const float scale = 1.f / sqrtf((float)hd);
  const long qs = (long)(H + 2 * G) * hd;
  dim3 grid(B * H), block(DEC_THREADS);
#define L_(TT, HDD) hipLaunchKernelGGL((attn_decode_k<TT, HDD, true>), grid, block, 0, s, (const TT*)qkv, (TT*)kc, \
                                       (TT*)vc, (TT*)out, H, G, Tmax, 0, scale, pos, qs)
  if (dt == DType::BF16) {
    if (hd == 128) L_(bf16_t, 128); else L_(bf16_t, 64);
  } else {
    if (hd == 128) L_(f16_t, 128); else L_(f16_t, 64);
  }
#undef L_
}

}  // namespace bllm
