// Token (+ learned position) embedding forward with fused dropout, and a deterministic
// backward.
//
// Replaces reference GPT2.py:100-113 (tok_emb + pos_emb + drop_emb) and Llama3.py:191
// (tok_emb).  Backward: instead of float atomics into a [V, d] table (order-dependent
// sums), the binding sorts the token ids once (rocPRIM radix sort via at::sort) and this
// kernel lets the FIRST position of every run of equal ids sum that run's gradient rows
// in fp32 and write the table row once — bitwise reproducible, no host sync, no [V, d]
// fp32 scratch.  Position-embedding grads sum the B rows that share a position.
#include "common.h"

namespace bllm {

BLLM_DEBUG_WORD(embedding)

template <typename T, int VEC>
__global__ __launch_bounds__(256) void emb_fwd_k(const int64_t* __restrict__ idx, const T* __restrict__ wte,
                                                 const T* __restrict__ wpe, T* __restrict__ out, long N, int d,
                                                 int T_, uint64_t seed, uint64_t offset, uint32_t thr,
                                                 float inv_keep, bool drop, long vocab) {
  const int dv = d / VEC;
  const long total = N * dv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / dv;
    const int c = (int)(i - r * dv) * VEC;
    long tok = idx[r];
    BLLM_DASSERT(tok >= 0 && tok < vocab, DBG_EMB_INDEX);
#ifdef BLLM_KERNEL_DEBUG
    tok = tok < 0 ? 0 : (tok >= vocab ? vocab - 1 : tok);  // keep the debug run in bounds
#endif
    VecN<T, VEC> a = ldv<T, VEC>(wte + tok * d + c), o;
    VecN<T, VEC> b;
    if (wpe) b = ldv<T, VEC>(wpe + (long)(r % T_) * d + c);
    uint32_t bits[VEC];
    if (drop) drop_bits_run<VEC>(seed, offset + (uint64_t)(r * d + c), bits);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float x = to_f(a.v[j]);
      if (wpe) x += to_f(b.v[j]);
      if (drop) x = (bits[j] >= thr) ? x * inv_keep : 0.f;
      o.v[j] = from_f<T>(x);
    }
    stv<T, VEC>(out + r * d + c, o);
  }
}

// One wave per (sorted position, 64*VEC-column slice); only the waves on a run head work.  A run
// is summed in sorted order (fixed -> reproducible), four rows per trip with their loads in
// flight together; row indices come 16 per vector load (broadcast by v_readlane) and the run's
// end 64 ids per ballot probe.  With a byte-level vocabulary (the offline tokenizer) a run is
// hundreds of rows long: the previous one-workgroup-per-run walk, one dependent scalar load per
// row, was latency bound.
__device__ __forceinline__ long lane_i64(long v, int src) {
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)(v & 0xffffffff), src);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), src);
  return (long)(((unsigned long)(unsigned)hi << 32) | (unsigned)lo);
}

template <typename T, int VEC>
__global__ __launch_bounds__(256) void emb_bwd_tok_k(const int64_t* __restrict__ sorted,
                                                     const int64_t* __restrict__ perm, const T* __restrict__ dx,
                                                     T* __restrict__ grad, long N, int d, bool accumulate) {
  const long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= N) return;
  const int64_t id = sorted[i];
  if (i > 0 && sorted[i - 1] == id) return;
  const int lane = threadIdx.x & 63;
  const int c = (blockIdx.y * 64 + lane) * VEC;
  const bool live = c < d;
  // run end: 64 sorted ids per probe, first mismatch by ballot
  long e = i + 1;
  for (;;) {
    const long k = e + lane;
    const uint64_t m = __builtin_amdgcn_ballot_w64(k >= N || sorted[k] != id);
    if (m) {
      e += __builtin_ctzll(m);
      break;
    }
    e += 64;
  }
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  for (long k0 = i; k0 < e; k0 += 16) {
    // 16 row indices in one vector load, broadcast by v_readlane; 4 row loads in flight
    const long pk = k0 + (lane & 15) < e ? (long)perm[k0 + (lane & 15)] : 0;
    const int n = e - k0 < 16 ? (int)(e - k0) : 16;
    int u = 0;
    for (; u + 4 <= n; u += 4) {
      VecN<T, VEC> v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (live) v[q] = ldv<T, VEC>(dx + lane_i64(pk, u + q) * d + c);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] += live ? to_f(v[q].v[j]) : 0.f;
    }
    for (; u < n; ++u) {
      if (!live) continue;
      VecN<T, VEC> v = ldv<T, VEC>(dx + lane_i64(pk, u) * d + c);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += to_f(v.v[j]);
    }
  }
  if (!live) return;
  T* g = grad + id * d + c;
  VecN<T, VEC> o;
  if (accumulate) {
    VecN<T, VEC> old = ldv<T, VEC>(g);
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] += to_f(old.v[j]);
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) o.v[j] = from_f<T>(acc[j]);
  stv<T, VEC>(g, o);
}

template <typename T, int VEC>
__global__ __launch_bounds__(256) void emb_bwd_pos_k(const T* __restrict__ dx, T* __restrict__ grad, int B,
                                                     int T_, int d, bool accumulate) {
  const int dv = d / VEC;
  const long total = (long)T_ * dv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int t = (int)(i / dv);
    const int c = (int)(i - (long)t * dv) * VEC;
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    for (int b = 0; b < B; ++b) {
      VecN<T, VEC> v = ldv<T, VEC>(dx + ((long)b * T_ + t) * d + c);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += to_f(v.v[j]);
    }
    T* g = grad + (long)t * d + c;
    if (accumulate) {
      VecN<T, VEC> old = ldv<T, VEC>(g);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += to_f(old.v[j]);
    }
    VecN<T, VEC> o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) o.v[j] = from_f<T>(acc[j]);
    stv<T, VEC>(g, o);
  }
}

#define EMB_VEC(T, d, ...)                                                         \
  if ((d) % (16 / sizeof(T)) == 0) { constexpr int VEC = 16 / sizeof(T); __VA_ARGS__; } \
  else { constexpr int VEC = 1; __VA_ARGS__; }

static inline int grid_of(long n) {
  long g = (n + 255) / 256;
  return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

void embedding_fwd(DType dt, const int64_t* idx, const void* wte, const void* wpe, void* out, long N, int d,
                   int T_, float p, uint64_t seed, uint64_t offset, long vocab, hipStream_t s) {
  const uint32_t thr = drop_threshold16(p);
  const float inv_keep = drop_inv_keep(p);
  BLLM_DISPATCH(dt, T, {
    EMB_VEC(T, d, {
      hipLaunchKernelGGL((emb_fwd_k<T, VEC>), dim3(grid_of(N * d / VEC)), dim3(256), 0, s, idx, (const T*)wte,
                         (const T*)wpe, (T*)out, N, d, T_, seed, offset, thr, inv_keep, p > 0.f, vocab);
    });
  });
}

void embedding_bwd_tok(DType dt, const int64_t* sorted, const int64_t* perm, const void* dx, void* grad, long N,
                       int d, bool accumulate, hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    EMB_VEC(T, d, {
      const dim3 grid((unsigned)((N + 3) / 4), (unsigned)ceil_div(d, 64 * VEC));
      hipLaunchKernelGGL((emb_bwd_tok_k<T, VEC>), grid, dim3(256), 0, s, sorted, perm, (const T*)dx, (T*)grad,
                         N, d, accumulate);
    });
  });
}

void embedding_bwd_pos(DType dt, const void* dx, void* grad, int B, int T_, int d, bool accumulate, hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    EMB_VEC(T, d, {
      hipLaunchKernelGGL((emb_bwd_pos_k<T, VEC>), dim3(grid_of((long)T_ * d / VEC)), dim3(256), 0, s,
                         (const T*)dx, (T*)grad, B, T_, d, accumulate);
    });
  });
}

}  // namespace bllm
