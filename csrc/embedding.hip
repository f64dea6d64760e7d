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

// Token-embedding backward, deterministic and independent of how skewed the ids are.  The
// sorted positions are cut into blocks of EMB_BLK; one wave per (block, 64*VEC-column slice)
// walks its block in sorted order (rows fetched 4 at a time, their indices 64 per vector load
// and broadcast by v_readlane) and cuts it into segments of equal id:
//   * a segment that is a whole run (it does not touch a neighbouring block's run) writes the
//     table row directly;
//   * the block's first segment, when its run started in an earlier block, goes to part[blk][0];
//     its last segment, when its run continues into the next block (and did not start earlier),
//     to part[blk][1] -- fp32 partial rows.
// A second pass finishes every run that crosses blocks from the block where it ends, adding the
// partials block by block backwards (fixed order: bitwise reproducible).  Byte-level ids (the
// offline tokenizer) make runs of thousands of rows -- the space character alone is ~15 % of
// the text -- which one wave per run walked in ~5 ms per step.
constexpr int EMB_BLK = 128;

__device__ __forceinline__ long lane_i64(long v, int src) {
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)(v & 0xffffffff), src);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), src);
  return (long)(((unsigned long)(unsigned)hi << 32) | (unsigned)lo);
}

template <typename T, int VEC>
__device__ __forceinline__ void emb_store_row(T* grad, long id, int d, int c, const float (&acc)[VEC], bool accumulate) {
  T* g = grad + id * d + c;
  float v[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) v[j] = acc[j];
  if (accumulate) {
    VecN<T, VEC> old = ldv<T, VEC>(g);
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] += to_f(old.v[j]);
  }
  VecN<T, VEC> o;
#pragma unroll
  for (int j = 0; j < VEC; ++j) o.v[j] = from_f<T>(v[j]);
  stv<T, VEC>(g, o);
}

template <typename T, int VEC>
__global__ __launch_bounds__(64) void emb_bwd_tok_k(const int64_t* __restrict__ sorted,
                                                    const int64_t* __restrict__ perm, const T* __restrict__ dx,
                                                    T* __restrict__ grad, float* __restrict__ part, long N, int d,
                                                    bool accumulate) {
  const int lane = threadIdx.x;
  const long k = blockIdx.x, b0 = k * EMB_BLK, b1 = b0 + EMB_BLK < N ? b0 + EMB_BLK : N;
  const int c = (blockIdx.y * 64 + lane) * VEC;
  const bool live = c < d;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  long cur = sorted[b0], s0 = b0;
  auto flush = [&](long s1) {  // segment [s0, s1) of id cur
    const bool before = s0 == b0 && b0 > 0 && sorted[b0 - 1] == cur;
    const bool after = s1 == b1 && b1 < N && sorted[b1] == cur;
    if (live) {
      if (!before && !after) {
        emb_store_row<T, VEC>(grad, cur, d, c, acc, accumulate);
      } else {
        float* pr = part + ((k * 2 + (before ? 0 : 1)) * (long)d + c);
#pragma unroll
        for (int j = 0; j < VEC; ++j) pr[j] = acc[j];
      }
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  };
  for (long p0 = b0; p0 < b1; p0 += 64) {
    const int n = b1 - p0 < 64 ? (int)(b1 - p0) : 64;
    const long myid = lane < n ? (long)sorted[p0 + lane] : -1;
    const long myrow = lane < n ? (long)perm[p0 + lane] : 0;
    for (int u = 0; u < n; u += 4) {
      VecN<T, VEC> v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (live && u + q < n) v[q] = ldv<T, VEC>(dx + lane_i64(myrow, u + q) * d + c);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (u + q >= n) break;
        const long id = lane_i64(myid, u + q);
        if (id != cur) {
          flush(p0 + u + q);
          cur = id;
          s0 = p0 + u + q;
        }
        if (live) {
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[j] += to_f(v[q].v[j]);
        }
      }
    }
  }
  flush(b1);
}

// runs that cross blocks, finished in the block where they end
template <typename T, int VEC>
__global__ __launch_bounds__(64) void emb_bwd_tok_fix_k(const int64_t* __restrict__ sorted,
                                                        T* __restrict__ grad, const float* __restrict__ part, long N,
                                                        int d, bool accumulate) {
  const long k = blockIdx.x, b0 = k * EMB_BLK, b1 = b0 + EMB_BLK < N ? b0 + EMB_BLK : N;
  if (k == 0) return;
  const long id = sorted[b0];
  if (sorted[b0 - 1] != id) return;                                        // no run enters the block
  if (sorted[b1 - 1] == id && b1 < N && sorted[b1] == id) return;          // it continues past it
  const int c = (blockIdx.y * 64 + threadIdx.x) * VEC;
  if (c >= d) return;
  float acc[VEC];
  const float* pr = part + (k * 2 + 0) * (long)d + c;
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = pr[j];
  for (long b = k - 1;; --b) {
    const long bs = b * EMB_BLK;
    const bool start = sorted[bs] != id || bs == 0 || sorted[bs - 1] != id;  // the run starts in block b
    const float* q = part + (b * 2 + (start ? 1 : 0)) * (long)d + c;
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] += q[j];
    if (start) break;
  }
  emb_store_row<T, VEC>(grad, id, d, c, acc, accumulate);
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

long embedding_bwd_part_floats(long N, int d) { return (long)ceil_div(N, EMB_BLK) * 2 * d; }

void embedding_bwd_tok(DType dt, const int64_t* sorted, const int64_t* perm, const void* dx, void* grad, float* part,
                       long N, int d, bool accumulate, hipStream_t s) {
  if (N <= 0) return;
  BLLM_DISPATCH(dt, T, {
    EMB_VEC(T, d, {
      const dim3 grid((unsigned)ceil_div(N, EMB_BLK), (unsigned)ceil_div(d, 64 * VEC));
      hipLaunchKernelGGL((emb_bwd_tok_k<T, VEC>), grid, dim3(64), 0, s, sorted, perm, (const T*)dx, (T*)grad, part,
                         N, d, accumulate);
      hipLaunchKernelGGL((emb_bwd_tok_fix_k<T, VEC>), grid, dim3(64), 0, s, sorted, (T*)grad, (const float*)part, N,
                         d, accumulate);
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
