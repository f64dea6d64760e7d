// Scalar (non-MFMA) causal attention forward/backward on the packed qkv layout.
//
// Role: the path for head dims the MFMA kernels do not tile (e.g. the reference's
// ``--debug`` model has head_dim 2, build_components.py:72-80) and an on-device oracle for
// the MFMA kernels.  One thread per query row (forward, dQ) or per key row (dK/dV), fp32
// registers, online softmax.  Same contract as attn_fwd.hip / attn_bwd.hip:
//   qkv [B*T, (H+2G)*hd]: q head h at col h*hd, k head g at (H+g)*hd, v head g at (H+G+g)*hd
//   o   [B*T, H*hd];  lse [B,H,T] = log2 sum_k exp2(s_qk * scale * log2e)
//   dropout keep(b,h,q,k) = hash(seed, offset + ((b*H+h)*T+q)*T+k) >= p*2^32
#include <float.h>
#include "api.h"

namespace bllm {

constexpr float LOG2E = 1.4426950408889634f;

template <typename T, int MAXD>
__global__ __launch_bounds__(64) void attn_fwd_naive_k(const T* __restrict__ qkv, T* __restrict__ o,
                                                       float* __restrict__ lse, int B, int T_, int H, int G, int hd,
                                                       bool causal, uint32_t thr, float inv_keep, bool drop,
                                                       uint64_t seed, uint64_t offset) {
  const long gid = blockIdx.x * 64L + threadIdx.x;
  if (gid >= (long)B * H * T_) return;
  const int q = (int)(gid % T_);
  const int h = (int)((gid / T_) % H);
  const int b = (int)(gid / ((long)T_ * H));
  const int g = h / (H / G);
  const long rs = (long)(H + 2 * G) * hd;
  const float c = rsqrtf((float)hd) * LOG2E;
  float qv[MAXD], acc[MAXD];
  const T* qp = qkv + ((long)b * T_ + q) * rs + (long)h * hd;
  for (int i = 0; i < hd; ++i) { qv[i] = to_f(qp[i]) * c; acc[i] = 0.f; }
  float m = -FLT_MAX, l = 0.f;
  const int kend = causal ? q + 1 : T_;
  for (int k = 0; k < kend; ++k) {
    const T* kp = qkv + ((long)b * T_ + k) * rs + (long)(H + g) * hd;
    const T* vp = qkv + ((long)b * T_ + k) * rs + (long)(H + G + g) * hd;
    float s = 0.f;
    for (int i = 0; i < hd; ++i) s += qv[i] * to_f(kp[i]);
    const float mn = fmaxf(m, s);
    const float alpha = exp2f(m - mn);
    const float pr = exp2f(s - mn);
    l = l * alpha + pr;
    float pw = pr;
    if (drop) pw = (drop_bits16(seed, offset + (((uint64_t)(b * H + h) * T_ + q) * T_ + k)) >= thr) ? pr * inv_keep : 0.f;
    for (int i = 0; i < hd; ++i) acc[i] = acc[i] * alpha + pw * to_f(vp[i]);
    m = mn;
  }
  T* op = o + ((long)b * T_ + q) * (long)H * hd + (long)h * hd;
  const float inv = 1.f / l;
  for (int i = 0; i < hd; ++i) op[i] = from_f<T>(acc[i] * inv);
  lse[((long)b * H + h) * T_ + q] = m + log2f(l);
}

// delta[b,h,q] = sum_i dO * O
template <typename T>
__global__ __launch_bounds__(256) void attn_delta_k(const T* __restrict__ o, const T* __restrict__ dout,
                                                    float* __restrict__ delta, int B, int T_, int H, int hd) {
  // one wave per (b, h, q)
  const long w = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= (long)B * H * T_) return;
  const int q = (int)(w % T_);
  const int h = (int)((w / T_) % H);
  const int b = (int)(w / ((long)T_ * H));
  const long off = ((long)b * T_ + q) * (long)H * hd + (long)h * hd;
  float s = 0.f;
  for (int i = lane; i < hd; i += 64) s += to_f(o[off + i]) * to_f(dout[off + i]);
  s = wave_sum(s);
  if (lane == 0) delta[((long)b * H + h) * T_ + q] = s;
}

template <typename T, int MAXD>
__global__ __launch_bounds__(64) void attn_bwd_dq_naive_k(const T* __restrict__ qkv, const float* __restrict__ lse,
                                                          const float* __restrict__ delta, const T* __restrict__ dout,
                                                          T* __restrict__ dqkv, int B, int T_, int H, int G, int hd,
                                                          bool causal, uint32_t thr, float inv_keep, bool drop,
                                                          uint64_t seed, uint64_t offset) {
  const long gid = blockIdx.x * 64L + threadIdx.x;
  if (gid >= (long)B * H * T_) return;
  const int q = (int)(gid % T_);
  const int h = (int)((gid / T_) % H);
  const int b = (int)(gid / ((long)T_ * H));
  const int g = h / (H / G);
  const long rs = (long)(H + 2 * G) * hd;
  const float scale = rsqrtf((float)hd), c = scale * LOG2E;
  float qv[MAXD], dov[MAXD], dq[MAXD];
  const T* qp = qkv + ((long)b * T_ + q) * rs + (long)h * hd;
  const T* dop = dout + ((long)b * T_ + q) * (long)H * hd + (long)h * hd;
  for (int i = 0; i < hd; ++i) { qv[i] = to_f(qp[i]); dov[i] = to_f(dop[i]); dq[i] = 0.f; }
  const float L = lse[((long)b * H + h) * T_ + q], D = delta[((long)b * H + h) * T_ + q];
  const int kend = causal ? q + 1 : T_;
  for (int k = 0; k < kend; ++k) {
    const T* kp = qkv + ((long)b * T_ + k) * rs + (long)(H + g) * hd;
    const T* vp = qkv + ((long)b * T_ + k) * rs + (long)(H + G + g) * hd;
    float s = 0.f, dp = 0.f;
    for (int i = 0; i < hd; ++i) { s += qv[i] * to_f(kp[i]); dp += dov[i] * to_f(vp[i]); }
    const float pr = exp2f(s * c - L);
    if (drop) dp = (drop_bits16(seed, offset + (((uint64_t)(b * H + h) * T_ + q) * T_ + k)) >= thr) ? dp * inv_keep : 0.f;
    const float ds = pr * (dp - D) * scale;
    for (int i = 0; i < hd; ++i) dq[i] += ds * to_f(kp[i]);
  }
  T* dqp = dqkv + ((long)b * T_ + q) * rs + (long)h * hd;
  for (int i = 0; i < hd; ++i) dqp[i] = from_f<T>(dq[i]);
}

template <typename T, int MAXD>
__global__ __launch_bounds__(64) void attn_bwd_dkv_naive_k(const T* __restrict__ qkv, const float* __restrict__ lse,
                                                           const float* __restrict__ delta, const T* __restrict__ dout,
                                                           T* __restrict__ dqkv, int B, int T_, int H, int G, int hd,
                                                           bool causal, uint32_t thr, float inv_keep, bool drop,
                                                           uint64_t seed, uint64_t offset) {
  const long gid = blockIdx.x * 64L + threadIdx.x;
  if (gid >= (long)B * G * T_) return;
  const int k = (int)(gid % T_);
  const int g = (int)((gid / T_) % G);
  const int b = (int)(gid / ((long)T_ * G));
  const int rep = H / G;
  const long rs = (long)(H + 2 * G) * hd;
  const float scale = rsqrtf((float)hd), c = scale * LOG2E;
  float kv[MAXD], vv[MAXD], dk[MAXD], dv[MAXD];
  const T* kp = qkv + ((long)b * T_ + k) * rs + (long)(H + g) * hd;
  const T* vp = qkv + ((long)b * T_ + k) * rs + (long)(H + G + g) * hd;
  for (int i = 0; i < hd; ++i) { kv[i] = to_f(kp[i]); vv[i] = to_f(vp[i]); dk[i] = 0.f; dv[i] = 0.f; }
  for (int r = 0; r < rep; ++r) {
    const int h = g * rep + r;
    for (int q = causal ? k : 0; q < T_; ++q) {
      const T* qp = qkv + ((long)b * T_ + q) * rs + (long)h * hd;
      const T* dop = dout + ((long)b * T_ + q) * (long)H * hd + (long)h * hd;
      float s = 0.f, dp = 0.f;
      for (int i = 0; i < hd; ++i) { s += to_f(qp[i]) * kv[i]; dp += to_f(dop[i]) * vv[i]; }
      const float L = lse[((long)b * H + h) * T_ + q], D = delta[((long)b * H + h) * T_ + q];
      const float pr = exp2f(s * c - L);
      float pd = pr;
      if (drop) {
        const bool keep = drop_bits16(seed, offset + (((uint64_t)(b * H + h) * T_ + q) * T_ + k)) >= thr;
        pd = keep ? pr * inv_keep : 0.f;
        dp = keep ? dp * inv_keep : 0.f;
      }
      const float ds = pr * (dp - D) * scale;
      for (int i = 0; i < hd; ++i) {
        dv[i] += pd * to_f(dop[i]);
        dk[i] += ds * to_f(qp[i]);
      }
    }
  }
  T* dkp = dqkv + ((long)b * T_ + k) * rs + (long)(H + g) * hd;
  T* dvp = dqkv + ((long)b * T_ + k) * rs + (long)(H + G + g) * hd;
  for (int i = 0; i < hd; ++i) { dkp[i] = from_f<T>(dk[i]); dvp[i] = from_f<T>(dv[i]); }
}

#define NAIVE_HD(hd, ...)                                   \
  if ((hd) <= 16) { constexpr int MAXD = 16; __VA_ARGS__; } \
  else if ((hd) <= 64) { constexpr int MAXD = 64; __VA_ARGS__; } \
  else if ((hd) <= 128) { constexpr int MAXD = 128; __VA_ARGS__; } \
  else { constexpr int MAXD = 256; __VA_ARGS__; }

void attn_fwd_naive(DType dt, const void* qkv, void* o, float* lse, int B, int T_, int H, int G, int hd, bool causal,
                    float p, uint64_t seed, uint64_t offset, hipStream_t s) {
  const uint32_t thr = drop_threshold16(p);
  const float ik = drop_inv_keep(p);
  const long n = (long)B * H * T_;
  BLLM_DISPATCH(dt, T, NAIVE_HD(hd, {
    hipLaunchKernelGGL((attn_fwd_naive_k<T, MAXD>), dim3(ceil_div(n, 64)), dim3(64), 0, s, (const T*)qkv, (T*)o,
                       lse, B, T_, H, G, hd, causal, thr, ik, p > 0.f, seed, offset);
  }));
}

void attn_delta(DType dt, const void* o, const void* dout, float* delta, int B, int T_, int H, int hd,
                hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    hipLaunchKernelGGL(attn_delta_k<T>, dim3(ceil_div((long)B * H * T_, 4)), dim3(256), 0, s, (const T*)o,
                       (const T*)dout, delta, B, T_, H, hd);
  });
}

void attn_bwd_naive(DType dt, const void* qkv, const void* o, const float* lse, const void* dout, void* dqkv,
                    float* delta, int B, int T_, int H, int G, int hd, bool causal, float p, uint64_t seed,
                    uint64_t offset, hipStream_t s) {
  const uint32_t thr = drop_threshold16(p);
  const float ik = drop_inv_keep(p);
  attn_delta(dt, o, dout, delta, B, T_, H, hd, s);
  BLLM_DISPATCH(dt, T, NAIVE_HD(hd, {
    hipLaunchKernelGGL((attn_bwd_dq_naive_k<T, MAXD>), dim3(ceil_div((long)B * H * T_, 64)), dim3(64), 0, s,
                       (const T*)qkv, lse, delta, (const T*)dout, (T*)dqkv, B, T_, H, G, hd, causal, thr, ik, p > 0.f,
                       seed, offset);
    hipLaunchKernelGGL((attn_bwd_dkv_naive_k<T, MAXD>), dim3(ceil_div((long)B * G * T_, 64)), dim3(64), 0, s,
                       (const T*)qkv, lse, delta, (const T*)dout, (T*)dqkv, B, T_, H, G, hd, causal, thr, ik, p > 0.f,
                       seed, offset);
  }));
}

}  // namespace bllm
