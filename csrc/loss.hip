// Fused cross-entropy forward / in-place backward over bf16/fp16/fp32 logits [N, V].
//
// Replaces reference train.py:88-92 (F.cross_entropy(logits.flatten(0,1), targets), mean
// over targets != -100).  One 256-thread workgroup per row; single pass online
// log-sum-exp (running max + rescaled sum per lane, combined across the workgroup), fp32
// math.  Backward overwrites the logits buffer with (softmax - onehot) * scale so the
// [N, V] gradient never needs a second allocation (1 GiB at Llama-3 vocab, N = 4096).
// Rows need not be 16-B aligned (GPT-2's V = 50257 is odd): scalar head/tail + vector body.
#include <float.h>
#include "common.h"

namespace bllm {

BLLM_DEBUG_WORD(loss)

template <typename T>
__device__ __forceinline__ void online_add(float x, float& m, float& s) {
  if (x > m) {
    s = s * __expf(m - x) + 1.f;
    m = x;
  } else {
    s += __expf(x - m);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_k(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                float* __restrict__ loss, float* __restrict__ lse_out, long V,
                                                long ld, long ignore_index) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float sm[4], ss[4];
  const long row = blockIdx.x;
  const T* p = logits + row * ld;
  const int mis = (int)(((uintptr_t)p / sizeof(T)) % VEC);
  const long head = mis ? (long)(VEC - mis) < V ? (VEC - mis) : V : 0;
  const long nv = (V - head) / VEC;
  const long tail0 = head + nv * VEC;
  float m = -FLT_MAX, s = 0.f;
  for (long i = threadIdx.x; i < head; i += 256) online_add<T>(to_f(p[i]), m, s);
  const T* pv = p + head;
  for (long i = threadIdx.x; i < nv; i += 256) {
    Vec16<T> r = ld16(pv + i * VEC);
    float vmax = to_f(r.v[0]);
#pragma unroll
    for (int j = 1; j < VEC; ++j) vmax = fmaxf(vmax, to_f(r.v[j]));
    if (vmax > m) {
      s *= __expf(m - vmax);
      m = vmax;
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) s += __expf(to_f(r.v[j]) - m);
  }
  for (long i = tail0 + threadIdx.x; i < V; i += 256) online_add<T>(to_f(p[i]), m, s);
  // combine (m, s) across the wave then across the 4 waves
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, mo);
    s = (m == -FLT_MAX ? 0.f : s * __expf(m - mn)) + (mo == -FLT_MAX ? 0.f : so * __expf(mo - mn));
    m = mn;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    float S = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) S += sm[i] == -FLT_MAX ? 0.f : ss[i] * __expf(sm[i] - M);
    const float l = M + __logf(S);
    lse_out[row] = l;
    long t = tgt[row];
    BLLM_DASSERT(t == ignore_index || (t >= 0 && t < V), DBG_CE_TARGET);
#ifdef BLLM_KERNEL_DEBUG
    if (t != ignore_index && (t < 0 || t >= V)) t = ignore_index;
#endif
    loss[row] = (t == ignore_index) ? 0.f : l - to_f(p[t]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_k(T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                const float* __restrict__ lse, const float* __restrict__ scale_p,
                                                long V, long ld, long ignore_index) {
  constexpr int VEC = 16 / sizeof(T);
  const long row = blockIdx.x;
  T* p = logits + row * ld;
  const long t = tgt[row];
  const bool valid = t != ignore_index;
  const float sc = valid ? scale_p[0] : 0.f;
  const float l = lse[row];
  const int mis = (int)(((uintptr_t)p / sizeof(T)) % VEC);
  const long head = mis ? ((long)(VEC - mis) < V ? (VEC - mis) : V) : 0;
  const long nv = (V - head) / VEC;
  const long tail0 = head + nv * VEC;
  for (long i = threadIdx.x; i < head; i += 256) p[i] = from_f<T>(__expf(to_f(p[i]) - l) * sc - (i == t ? sc : 0.f));
  T* pv = p + head;
  for (long i = threadIdx.x; i < nv; i += 256) {
    Vec16<T> r = ld16(pv + i * VEC);
    const long c0 = head + i * VEC;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float g = __expf(to_f(r.v[j]) - l) * sc;
      if (c0 + j == t) g -= sc;
      r.v[j] = from_f<T>(g);
    }
    st16(pv + i * VEC, r);
  }
  for (long i = tail0 + threadIdx.x; i < V; i += 256) p[i] = from_f<T>(__expf(to_f(p[i]) - l) * sc - (i == t ? sc : 0.f));
}

// rows ld elements apart (ld > V: the vocabulary padded to whole GEMM tiles, pad columns untouched)
void ce_fwd(DType dt, const void* logits, const int64_t* tgt, float* loss, float* lse, long N, long V, long ld,
            long ignore_index, hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    hipLaunchKernelGGL(ce_fwd_k<T>, dim3(N), dim3(256), 0, s, (const T*)logits, tgt, loss, lse, V, ld, ignore_index);
  });
}
void ce_bwd(DType dt, void* logits, const int64_t* tgt, const float* lse, const float* scale, long N, long V, long ld,
            long ignore_index, hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    hipLaunchKernelGGL(ce_bwd_k<T>, dim3(N), dim3(256), 0, s, (T*)logits, tgt, lse, scale, V, ld, ignore_index);
  });
}

}  // namespace bllm
