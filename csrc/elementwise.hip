// Elementwise kernels: SwiGLU, exact-erf GELU, dropout(+residual), RoPE.
//
// Replaces reference common_components.py:6-35 (RoPE), :78-124 (SiLU/SwiGLU),
// GPT2.py:58-62 (nn.GELU, exact erf), and nn.Dropout.  All are HBM-bound: 16-byte
// accesses per lane, grid-stride loops capped at 256 CUs x 8 workgroups.
#include <cstdlib>
#include "api.h"

namespace bllm {

BLLM_DEBUG_WORD(elementwise)

static inline int ew_grid(long nvec) {
  long g = (nvec + 255) / 256;
  return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

// ---------------------------------------------------------------- SwiGLU
// gu: [N, 2F] = [gate | up] per row (fused [fc1; fc2] GEMM output); act: [N, F]
template <typename T, int VEC>
__global__ __launch_bounds__(256) void swiglu_fwd_k(const T* __restrict__ gu, T* __restrict__ act, long N, int F,
                                                    long lda) {
  const int fv = F / VEC;
  const long total = N * fv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / fv;
    const int c = (int)(i - r * fv) * VEC;
    VecN<T, VEC> g = ldv<T, VEC>(gu + r * 2 * F + c), u = ldv<T, VEC>(gu + r * 2 * F + F + c), o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float a = to_f(g.v[j]);
      o.v[j] = from_f<T>(a * silu_sig(a) * to_f(u.v[j]));
    }
    stv<T, VEC>(act + r * lda + c, o);
  }
}

template <typename T, int VEC>
__global__ __launch_bounds__(256) void swiglu_bwd_k(const T* __restrict__ gu, const T* dact,
                                                    T* __restrict__ dgu, T* act, long N, int F) {
  const int fv = F / VEC;
  const long total = N * fv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / fv;
    const int c = (int)(i - r * fv) * VEC;
    VecN<T, VEC> g = ldv<T, VEC>(gu + r * 2 * F + c), u = ldv<T, VEC>(gu + r * 2 * F + F + c), d = ldv<T, VEC>(dact + r * F + c);
    VecN<T, VEC> dg, du, o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float a = to_f(g.v[j]), b = to_f(u.v[j]), dd = to_f(d.v[j]);
      const float sg = silu_sig(a);
      dg.v[j] = from_f<T>(dd * b * sg * (1.f + a * (1.f - sg)));
      du.v[j] = from_f<T>(dd * a * sg);
      o.v[j] = from_f<T>(a * sg * b);  // bitwise as swiglu_fwd
    }
    stv<T, VEC>(dgu + r * 2 * F + c, dg);
    stv<T, VEC>(dgu + r * 2 * F + F + c, du);
    if (act) stv<T, VEC>(act + r * F + c, o);
  }
}

// SwiGLU backward whose incoming gradient is the down projection's K-augmented LoRA dX:
//   dact = base + s . u P      (base = dy W from the dX GEMM, u = dy B^T [N, r], P = A^T [r, F])
// is formed on the fly instead of by a read-modify-write pass over [N, F] (lora_up).  A workgroup
// owns LR_ROWS rows: their u rows sit in LDS, and each thread keeps the r x 8 slice of P for its
// column vector in registers across the rows, so P is read once per workgroup, not per row.
constexpr int LR_ROWS = 16;
template <typename T, int R>
__global__ __launch_bounds__(256) void swiglu_bwd_lr_k(const T* __restrict__ gu, const T* __restrict__ base,
                                                       long ldb, const T* __restrict__ u, long ldu,
                                                       const T* __restrict__ P, float s, T* __restrict__ dgu,
                                                       long N, int F) {
  constexpr int VEC = 8;
  __shared__ float us[LR_ROWS][R];
  const long r0 = (long)blockIdx.x * LR_ROWS;
  for (int e = threadIdx.x; e < LR_ROWS * R; e += 256) {
    const int rr = e / R, j = e - rr * R;
    us[rr][j] = r0 + rr < N ? to_f(u[(r0 + rr) * ldu + j]) : 0.f;
  }
  __syncthreads();
  const int fv = F / VEC;
  for (int cv = threadIdx.x; cv < fv; cv += 256) {
    const int c = cv * VEC;
    float pr[R][VEC];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const VecN<T, VEC> pv = ldv<T, VEC>(P + (long)j * F + c);
#pragma unroll
      for (int e = 0; e < VEC; ++e) pr[j][e] = to_f(pv.v[e]);
    }
    for (int rr = 0; rr < LR_ROWS; ++rr) {
      const long r = r0 + rr;
      if (r >= N) break;
      const VecN<T, VEC> g = ldv<T, VEC>(gu + r * 2 * F + c), up = ldv<T, VEC>(gu + r * 2 * F + F + c);
      const VecN<T, VEC> bs = ldv<T, VEC>(base + r * ldb + c);
      float corr[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) corr[e] = 0.f;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const float uj = us[rr][j];
#pragma unroll
        for (int e = 0; e < VEC; ++e) corr[e] = fmaf(uj, pr[j][e], corr[e]);
      }
      VecN<T, VEC> dg, du;
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        // rounded to T like the lora_up output it replaces
        const float dd = to_f(from_f<T>(to_f(bs.v[e]) + s * corr[e]));
        const float a = to_f(g.v[e]), b = to_f(up.v[e]);
        const float sg = silu_sig(a);
        dg.v[e] = from_f<T>(dd * b * sg * (1.f + a * (1.f - sg)));
        du.v[e] = from_f<T>(dd * a * sg);
      }
      stv<T, VEC>(dgu + r * 2 * F + c, dg);
      stv<T, VEC>(dgu + r * 2 * F + F + c, du);
    }
  }
}

// SwiGLU backward of a LoRA MLP (K-augmented gate/up group + down projection, r = 16) with the
// three rank-16 weight-gradient reductions that read these rows fused into the same pass:
//   dact = base + s . u P;  (dg, du) = swiglu_bwd(gu, dact)                 (as swiglu_bwd_lr_k)
//   G0[j][c] = sum_n st[n][j]      . dg[n][c]      dB of the gate LoRA   (st = s t, gate | up)
//   G1[j][c] = sum_n st[n][16 + j] . du[n][c]      dB of the up LoRA
//   G2[j][c] = s sum_n u[n][j]     . act[n][c]     dA^T of the down LoRA (act = silu(g) up)
// -- the separate lora_wgrad passes re-read dgu ([N, 2F]) and act ([N, F]) from HBM.  Column-slab
// mapping: a workgroup owns LRW_COLS columns of F and one of S contiguous row ranges, walked in
// LRW_CH-row chunks; thread (row rr, vector cv) computes 8 columns of one row as swiglu_bwd_lr_k
// (the P slice in registers), the chunk's dg / du / act (rounded as stored) and its st / u rows
// go through LDS, and the four waves run the reductions as 16x16x32 MFMAs (wave w: columns
// 16w .. 16w+15; both operands read with ds_read_b64_tr_b16, k = the chunk's rows).  fp32
// partials per row range [S][3][16][F] are summed by lora_reduce (fixed order: deterministic).
constexpr int LRW_COLS = 64, LRW_CH = 32;
constexpr int LRW_RS = LRW_COLS * 2 + 16;  // bytes per row of a dg / du / act tile (padded)
constexpr int LRW_LS = 32;                 // bytes per row of an st / u tile (16 x 16-bit)

typedef short lrw_s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) lrw_s16x4 lrw_lds_s16x4;
typedef float lrw_f32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct LrwMfma;
template <> struct LrwMfma<bf16_t> {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ lrw_f32x4 run(v8 a, v8 b, lrw_f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct LrwMfma<f16_t> {
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ lrw_f32x4 run(v8 a, v8 b, lrw_f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
// 8 k-values (rows 8g .. 8g+7 of a tile) of one column for this lane: two transposed reads
template <typename v8>
__device__ __forceinline__ v8 lrw_frag(const char* tile, int stride, int col_byte, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const char* a = tile + (8 * g + q) * stride + col_byte + 8 * p;
  const lrw_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lrw_lds_s16x4*)(a));
  const lrw_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lrw_lds_s16x4*)(a + 4 * stride));
  return __builtin_bit_cast(v8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <typename T>
__global__ __launch_bounds__(256, 2) void swiglu_bwd_lr_wg_k(const T* __restrict__ gu, const T* __restrict__ base,
                                                          long ldb, const T* __restrict__ u, long ldu,
                                                          const T* __restrict__ P, const T* __restrict__ st,
                                                          long ldst, float s, T* __restrict__ dgu,
                                                          float* __restrict__ part, long N, int F, long rows_per) {
  constexpr int R = 16, VEC = 8;
  typedef typename LrwMfma<T>::v8 v8;
  __shared__ __attribute__((aligned(16))) char Lt[2][3][LRW_CH * LRW_LS];  // st gate, st up, u
  __shared__ __attribute__((aligned(16))) char Rt[2][3][LRW_CH * LRW_RS];  // dg, du, act
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rr = tid >> 3, cv = tid & 7;
  const int c = blockIdx.x * LRW_COLS + cv * VEC;
  const long r0 = (long)blockIdx.y * rows_per;
  const long r1 = r0 + rows_per < N ? r0 + rows_per : N;

  float pr[R][VEC];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const Vec16<T> pv = ld16(P + (long)j * F + c);
#pragma unroll
    for (int e = 0; e < VEC; ++e) pr[j][e] = to_f(pv.v[e]);
  }
  // st / u staging: thread t < 192 moves 16 B = half a 16-wide row of tile lq
  const int lq = tid >> 6, lrow = (tid & 63) >> 1, lh = tid & 1;
  const T* lsrc = lq == 0 ? st + 8 * lh : lq == 1 ? st + 16 + 8 * lh : u + 8 * lh;
  const long lld = lq == 2 ? ldu : ldst;

  Vec16<T> g, up, bs;
  uint4 lreg = make_uint4(0, 0, 0, 0);
  // per-thread row pointers, advanced by one chunk per load (no 64-bit multiplies in the loop)
  const T* pg = gu + (r0 + rr) * 2 * F + c;
  const T* pb = base + (r0 + rr) * ldb + c;
  const T* pl = lsrc + (r0 + lrow) * lld;
  T* pd = dgu + (r0 + rr) * 2 * F + c;
  const long step_g = (long)LRW_CH * 2 * F, step_b = (long)LRW_CH * ldb, step_l = (long)LRW_CH * lld;
  auto load = [&](long row) {
    if (row + rr < r1) {
      g = ld16(pg);
      up = ld16(pg + F);
      bs = ld16(pb);
    }
    lreg = make_uint4(0, 0, 0, 0);
    if (lq < 3 && row + lrow < r1) lreg = *reinterpret_cast<const uint4*>(pl);
    pg += step_g, pb += step_b, pl += step_l;
  };
  lrw_f32x4 acc[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) acc[q] = lrw_f32x4{0.f, 0.f, 0.f, 0.f};
  if (r0 < r1) load(r0);
  int par = 0;
  for (long row = r0; row < r1; row += LRW_CH, par ^= 1) {
    if (lq < 3) *reinterpret_cast<uint4*>(Lt[par][lq] + lrow * LRW_LS + lh * 16) = lreg;
    __syncthreads();  // st / u rows of this chunk visible (and the chunk before last's tiles free)
    const bool valid = row + rr < r1;
    const Vec16<T> cg = g, cu = up, cb = bs;
    if (row + LRW_CH < r1) load(row + LRW_CH);  // next chunk's loads in flight under the math
    float uj[R];
    {
      const Vec16<T> u0 = ld16(reinterpret_cast<const T*>(Lt[par][2] + rr * LRW_LS));
      const Vec16<T> u1 = ld16(reinterpret_cast<const T*>(Lt[par][2] + rr * LRW_LS + 16));
#pragma unroll
      for (int e = 0; e < VEC; ++e) uj[e] = to_f(u0.v[e]), uj[VEC + e] = to_f(u1.v[e]);
    }
    Vec16<T> dg, du, act;
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      float corr = 0.f;
#pragma unroll
      for (int j = 0; j < R; ++j) corr = fmaf(uj[j], pr[j][e], corr);
      // rounded to T like the lora_up output it replaces (as swiglu_bwd_lr_k)
      const float dd = to_f(from_f<T>(to_f(cb.v[e]) + s * corr));
      const float a = to_f(cg.v[e]), b = to_f(cu.v[e]);
      const float sg = silu_sig(a);
      dg.v[e] = valid ? from_f<T>(dd * b * sg * (1.f + a * (1.f - sg))) : from_f<T>(0.f);
      du.v[e] = valid ? from_f<T>(dd * a * sg) : from_f<T>(0.f);
      act.v[e] = valid ? from_f<T>(a * sg * b) : from_f<T>(0.f);  // bitwise as swiglu_fwd
    }
    if (valid) {
      st16(pd, dg);
      st16(pd + F, du);
    }
    pd += step_g;
    st16(reinterpret_cast<T*>(Rt[par][0] + rr * LRW_RS + cv * 16), dg);
    st16(reinterpret_cast<T*>(Rt[par][1] + rr * LRW_RS + cv * 16), du);
    st16(reinterpret_cast<T*>(Rt[par][2] + rr * LRW_RS + cv * 16), act);
    __syncthreads();  // the chunk's dg / du / act tiles visible
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const v8 a = lrw_frag<v8>(Lt[par][q], LRW_LS, 0, lane);
      const v8 b = lrw_frag<v8>(Rt[par][q], LRW_RS, 32 * w, lane);
      acc[q] = LrwMfma<T>::run(a, b, acc[q]);
    }
  }
  // C map of 16x16x32: column = lane & 15, rows 4 (lane >> 4) + i  ->  G_q[j][col]
  const int col = blockIdx.x * LRW_COLS + 16 * w + (lane & 15);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    float* o = part + ((long)blockIdx.y * 3 + q) * R * F + col;
    const float sc = q == 2 ? s : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[(long)(4 * (lane >> 4) + i) * F] = sc * acc[q][i];
  }
}

// Row-per-workgroup variants for wide FFNs (F/VEC >= 512, e.g. Llama F=14336): no 64-bit index
// division, U independent 16-B load pairs in flight per lane before any math (the grid-stride loop
// above serialises load -> compute per vector).  One workgroup per token row; N rows >> 256 CUs.
template <typename T, int VEC, int U>
__global__ __launch_bounds__(256) void swiglu_fwd_rows_k(const T* __restrict__ gu, T* __restrict__ act, int F,
                                                         long lda) {
  const int fv = F / VEC;
  const T* g0 = gu + (long)blockIdx.x * 2 * F;
  const T* u0 = g0 + F;
  T* o0 = act + (long)blockIdx.x * lda;
  for (int base = threadIdx.x; base < fv; base += 256 * U) {
    VecN<T, VEC> g[U], u[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int c = base + k * 256;
      if (c < fv) {
        g[k] = ldv<T, VEC>(g0 + c * VEC);
        u[k] = ldv<T, VEC>(u0 + c * VEC);
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int c = base + k * 256;
      if (c < fv) {
        VecN<T, VEC> o;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float a = to_f(g[k].v[j]);
          o.v[j] = from_f<T>(a * silu_sig(a) * to_f(u[k].v[j]));
        }
        stv<T, VEC>(o0 + c * VEC, o);
      }
    }
  }
}

template <typename T, int VEC, int U>
__global__ __launch_bounds__(256) void swiglu_bwd_rows_k(const T* __restrict__ gu, const T* dact,
                                                         T* __restrict__ dgu, T* act, int F) {
  const int fv = F / VEC;
  const long row = blockIdx.x;
  const T* g0 = gu + row * 2 * F;
  const T* u0 = g0 + F;
  const T* d0 = dact + row * F;
  T* dg0 = dgu + row * 2 * F;
  T* du0 = dg0 + F;
  T* a0 = act ? act + row * F : nullptr;
  for (int base = threadIdx.x; base < fv; base += 256 * U) {
    VecN<T, VEC> g[U], u[U], d[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int c = base + k * 256;
      if (c < fv) {
        g[k] = ldv<T, VEC>(g0 + c * VEC);
        u[k] = ldv<T, VEC>(u0 + c * VEC);
        d[k] = ldv<T, VEC>(d0 + c * VEC);
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int c = base + k * 256;
      if (c < fv) {
        VecN<T, VEC> dg, du, o;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float a = to_f(g[k].v[j]), b = to_f(u[k].v[j]), dd = to_f(d[k].v[j]);
          const float sg = silu_sig(a);
          dg.v[j] = from_f<T>(dd * b * sg * (1.f + a * (1.f - sg)));
          du.v[j] = from_f<T>(dd * a * sg);
          o.v[j] = from_f<T>(a * sg * b);  // bitwise as swiglu_fwd
        }
        stv<T, VEC>(dg0 + c * VEC, dg);
        stv<T, VEC>(du0 + c * VEC, du);
        if (a0) stv<T, VEC>(a0 + c * VEC, o);
      }
    }
  }
}

// ---------------------------------------------------------------- GELU (erf)
template <typename T, int VEC>
__global__ __launch_bounds__(256) void gelu_fwd_k(const T* __restrict__ f, T* __restrict__ g, long nvec) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nvec; i += (long)gridDim.x * 256) {
    VecN<T, VEC> a = ldv<T, VEC>(f + i * VEC), o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float x = to_f(a.v[j]);
      o.v[j] = from_f<T>(gelu_fwd_f<T>(x));
    }
    stv<T, VEC>(g + i * VEC, o);
  }
}

template <typename T, int VEC>
__global__ __launch_bounds__(256) void gelu_bwd_k(const T* __restrict__ f, const T* __restrict__ dg,
                                                  T* __restrict__ df, long nvec) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nvec; i += (long)gridDim.x * 256) {
    VecN<T, VEC> a = ldv<T, VEC>(f + i * VEC), d = ldv<T, VEC>(dg + i * VEC), o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float x = to_f(a.v[j]);
      o.v[j] = from_f<T>(to_f(d.v[j]) * gelu_grad(x));
    }
    stv<T, VEC>(df + i * VEC, o);
  }
}

// ---------------------------------------------------------------- dropout
// out = x + a * keep / (1-p)    (x may be null -> out = dropout(a))
template <typename T, int VEC>
__global__ __launch_bounds__(256) void dropout_add_k(const T* __restrict__ x, const T* __restrict__ a,
                                                     T* __restrict__ out, long nvec, uint64_t seed,
                                                     uint64_t offset, uint32_t thr, float inv_keep) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nvec; i += (long)gridDim.x * 256) {
    VecN<T, VEC> av = ldv<T, VEC>(a + i * VEC), o;
    VecN<T, VEC> xv;
    if (x) xv = ldv<T, VEC>(x + i * VEC);
    uint32_t bits[VEC];
    drop_bits_run<VEC>(seed, offset + (uint64_t)(i * VEC), bits);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const bool keep = bits[j] >= thr;
      float r = keep ? to_f(av.v[j]) * inv_keep : 0.f;
      if (x) r += to_f(xv.v[j]);
      o.v[j] = from_f<T>(r);
    }
    stv<T, VEC>(out + i * VEC, o);
  }
}

// ---------------------------------------------------------------- RoPE in place
// qkv [N, (H+2G)*hd]; rotates heads [0, H+G) of every row; position = row % T + pos_offset.
// One thread = 8 consecutive pairs (x1[i..i+7], x2[i..i+7]); cos/sin fp32 [Tctx, hd/2].
template <typename T>
__global__ __launch_bounds__(256) void rope_k(T* __restrict__ qkv, const float* __restrict__ cosT,
                                              const float* __restrict__ sinT, long N, int T_, int nh_rot,
                                              int row_stride, int hd, int pos_offset, float sgn,
                                              const int* __restrict__ pos_dev) {
  // one thread = 8 rotation pairs (two 16-B vectors of the head, 8 fp32 cos/sin each);
  // 32-bit index math (N * heads * chunks < 2^31 for every supported shape)
  static_assert(sizeof(T) == 2, "16-bit element types (fp32 uses rope_scalar_k)");
  const int half = hd / 2;
  if (pos_dev) {
    BLLM_DASSERT(*pos_dev >= 0, DBG_ROPE_POS);
    pos_offset += *pos_dev;
  }  // graph-replayed decode: position read at run time
  const int cpb = half / 8;  // chunks of 8 pairs per head
  const int per_row = nh_rot * cpb;
  const int total = (int)(N * per_row);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int r = i / per_row;
    const int rem = i - r * per_row;
    const int h = rem / cpb, ch = rem - h * cpb;
    const int pos = r % T_ + pos_offset;
    T* base = qkv + (long)r * row_stride + h * hd + ch * 8;
    const float* cp = cosT + (long)pos * half + ch * 8;
    const float* sp = sinT + (long)pos * half + ch * 8;
    const Vec16<T> a = ld16(base), b = ld16(base + half);
    const float4 c0 = *reinterpret_cast<const float4*>(cp), c1 = *reinterpret_cast<const float4*>(cp + 4);
    const float4 s0 = *reinterpret_cast<const float4*>(sp), s1 = *reinterpret_cast<const float4*>(sp + 4);
    const float c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    Vec16<T> oa, ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x1 = to_f(a.v[j]), x2 = to_f(b.v[j]), sj = sgn * sn[j];
      oa.v[j] = from_f<T>(x1 * c[j] - x2 * sj);
      ob.v[j] = from_f<T>(x2 * c[j] + x1 * sj);
    }
    st16(base, oa);
    st16(base + half, ob);
  }
}

// scalar fallback for head dims not multiple of 16
template <typename T>
__global__ __launch_bounds__(256) void rope_scalar_k(T* __restrict__ qkv, const float* __restrict__ cosT,
                                                     const float* __restrict__ sinT, long N, int T_, int nh_rot,
                                                     int row_stride, int hd, int pos_offset, float sgn,
                                                     const int* __restrict__ pos_dev) {
  const int half = hd / 2;
  if (pos_dev) {
    BLLM_DASSERT(*pos_dev >= 0, DBG_ROPE_POS);
    pos_offset += *pos_dev;
  }
  const long total = N * nh_rot * half;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int k = (int)(i % half);
    const long t = i / half;
    const int h = (int)(t % nh_rot);
    const long r = t / nh_rot;
    const int pos = (int)(r % T_) + pos_offset;
    T* base = qkv + r * row_stride + (long)h * hd;
    const float c = cosT[(long)pos * half + k], s = sgn * sinT[(long)pos * half + k];
    const float a = to_f(base[k]), b = to_f(base[half + k]);
    base[k] = from_f<T>(a * c - b * s);
    base[half + k] = from_f<T>(b * c + a * s);
  }
}

// Bias gradient db[f] (+)= sum_n dy[n, f]: replaces the eager column reduction of the GPT-2
// bias grads (reference nn.Linear bias).  Pass 1: workgroup (x = 256 threads x 8-column
// vectors, y = a row band) writes fp32 partial sums; pass 2 sums the bands in a fixed order and
// writes / accumulates the gradient in its dtype (deterministic, no atomics).
// row bands: narrow outputs (F <= 2048, e.g. GPT-2's 1280-wide biases: one 160-lane workgroup
// per band) get 4x more bands so enough waves stream dy; partials stay small (1024 x F fp32)
int colsum_bands(int N, int F) {
  const int cap = F <= 2048 ? 1024 : 256;
  return N >= 16 * cap ? cap : (N + 15) / 16;
}

// Elementwise backward + bias-gradient column sums in one pass (GPT-2: the dropout backward in
// front of the out_proj / c_proj bias grads, the GELU backward in front of the c_fc bias grad,
// reference GPT2.py:58-62 + nn.Linear bias).  Same band split, per-lane row order and fp32
// partials as the plain column sum (OP 3, bias_grad) over the rounded outputs, so db is bitwise
// the separate path's; the separate colsum pass's re-read of the [N, F] gradient is gone.
//   OP 0: out = dropout_bwd(src)  (keep bits by the counter hash at element index r * F + c)
//   OP 1: out = src * gelu'(aux)   (exact erf GELU); with act, also act = gelu(aux), bitwise as
//         gelu_fwd_k (act may alias src: the activation-checkpoint recompute of GPT-2 then
//         needs no GELU forward pass for the c_proj dW)
//   OP 3: column sums of src only (bias_grad: nothing stored but the partials)
// part == nullptr: no column sums (frozen / absent bias).
// OP 2 = OP 1 that also writes the activation (act != nullptr), a separate instantiation so the
// erff of that rebuild is not branched around per element when there is none.
// Mapping: each wave owns 64 column vectors (no partially filled workgroups at F = 1280 / 5120
// bf16) and one quarter of the band's rows (rows r0 + w, r0 + w + 4, ...); the next group of
// BR rows is loaded before the current one is processed (register double buffer), so every wave
// keeps 2 x BR x (1 or 2) 16-B loads in flight instead of draining between groups (the
// load-all / compute / store loop ran GPT2-774M's c_fc GELU backward at ~3 TB/s).  The four
// waves' column sums meet in LDS; one fp32 partial row per band as before.
template <typename T, int OP>
__global__ __launch_bounds__(256) void bwd_colsum_k(const T* src, const T* __restrict__ aux,
                                                    T* __restrict__ out, float* __restrict__ part, int N, int F,
                                                    int rows_per, uint64_t seed, uint64_t offset, uint32_t thr,
                                                    float inv_keep, T* act) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int BR = 4;                      // rows per group per wave
  constexpr bool AUX = OP == 1 || OP == 2;
  __shared__ float red[4][64 * VEC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cv = blockIdx.x * 64 + lane;
  const bool on = cv * VEC < F;
  const int r0 = blockIdx.y * rows_per, r1 = min(N, r0 + rows_per);
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  auto row = [&](int r, const Vec16<T>& v, const Vec16<T>& a) {
    const long e = (long)r * F + cv * VEC;
    Vec16<T> o;
    if constexpr (OP == 3) {
      o = v;
    } else if constexpr (OP == 0) {
      uint32_t bits[VEC];
      drop_bits_run<VEC>(seed, offset + (uint64_t)e, bits);
#pragma unroll
      for (int j = 0; j < VEC; ++j) o.v[j] = from_f<T>(bits[j] >= thr ? to_f(v.v[j]) * inv_keep : 0.f);
    } else {
      Vec16<T> g;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float x = to_f(a.v[j]);
        o.v[j] = from_f<T>(to_f(v.v[j]) * gelu_grad(x));
        if constexpr (OP == 2) g.v[j] = from_f<T>(gelu_fwd_f<T>(x));   // = gelu_fwd
      }
      if constexpr (OP == 2) st16(act + e, g);
    }
    if constexpr (OP != 3) st16(out + e, o);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      // opaque copy: for fp32 (from_f = identity) the compiler would otherwise fuse the output
      // product into the column sum (one FMA), skipping the rounding the stored output had --
      // the sums are over the stored (rounded) values, as the plain column sum (OP 3)
      float ov = to_f(o.v[j]);
      asm volatile("" : "+v"(ov));
      acc[j] += ov;
    }
  };
  if (on) {
    Vec16<T> v[BR], a[BR], vn[BR], an[BR];
    auto load = [&](int rb, Vec16<T> (&dv)[BR], Vec16<T> (&da)[BR]) {
#pragma unroll
      for (int k = 0; k < BR; ++k) {
        const int r = rb + 4 * k;            // wave-uniform
        if (r < r1) {
          dv[k] = ld16(src + (long)r * F + cv * VEC);
          if constexpr (AUX) da[k] = ld16(aux + (long)r * F + cv * VEC);
        }
      }
    };
    int rb = r0 + w;
    if (rb < r1) load(rb, v, a);
    while (rb < r1) {
      const int rn = rb + 4 * BR;
      if (rn < r1) load(rn, vn, an);
#pragma unroll
      for (int k = 0; k < BR; ++k)
        if (rb + 4 * k < r1) row(rb + 4 * k, v[k], a[k]);
#pragma unroll
      for (int k = 0; k < BR; ++k) {
        v[k] = vn[k];
        if constexpr (AUX) a[k] = an[k];
      }
      rb = rn;
    }
  }
  if (!part) return;
#pragma unroll
  for (int j = 0; j < VEC; ++j) red[w][lane * VEC + j] = acc[j];
  __syncthreads();
  if (w == 0 && on) {
    float* o = part + (long)blockIdx.y * F + cv * VEC;
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = ((red[0][lane * VEC + j] + red[1][lane * VEC + j]) + red[2][lane * VEC + j]) +
                                         red[3][lane * VEC + j];
  }
}

void bwd_bias_grad(DType dt, DType odt, int op, const void* src, const void* aux, void* out, float* part, void* db,
                   int N, int F, bool accumulate, float p, uint64_t seed, uint64_t offset, void* act, hipStream_t s) {
  const int P = colsum_bands(N, F);
  const int rows_per = (N + P - 1) / P;
  const uint32_t thr = drop_threshold16(p);
  const float inv_keep = drop_inv_keep(p);
  BLLM_DISPATCH(dt, T, {
    constexpr int VEC = 16 / sizeof(T);
    dim3 grid((F / VEC + 63) / 64, P);
    if (op == 0)
      hipLaunchKernelGGL((bwd_colsum_k<T, 0>), grid, dim3(256), 0, s, (const T*)src, (const T*)aux, (T*)out, part, N, F,
                         rows_per, seed, offset, thr, inv_keep, (T*)nullptr);
    else
      if (act)
        hipLaunchKernelGGL((bwd_colsum_k<T, 2>), grid, dim3(256), 0, s, (const T*)src, (const T*)aux, (T*)out, part, N,
                           F, rows_per, seed, offset, thr, inv_keep, (T*)act);
      else
        hipLaunchKernelGGL((bwd_colsum_k<T, 1>), grid, dim3(256), 0, s, (const T*)src, (const T*)aux, (T*)out, part, N,
                           F, rows_per, seed, offset, thr, inv_keep, (T*)nullptr);
  });
  if (part) col_reduce(part, odt, db, P, F, accumulate, s);
}

// dy [N, F] (F % (16/sizeof(T)) == 0), out [F] in dtype odt (written, or added when accumulate)
void bias_grad(DType dt, DType odt, const void* dy, float* part, void* out, int N, int F, bool accumulate,
               hipStream_t s) {
  const int P = colsum_bands(N, F);
  const int rows_per = (N + P - 1) / P;
  BLLM_DISPATCH(dt, T, {
    constexpr int VEC = 16 / sizeof(T);
    dim3 grid((F / VEC + 63) / 64, P);
    hipLaunchKernelGGL((bwd_colsum_k<T, 3>), grid, dim3(256), 0, s, (const T*)dy, (const T*)nullptr, (T*)nullptr,
                       part, N, F, rows_per, 0ull, 0ull, 0u, 0.f, (T*)nullptr);
  });
  col_reduce(part, odt, out, P, F, accumulate, s);
}

// ----------------------------------------------------------------------------- launchers
// VEC = 16 bytes per lane when the sizes allow it, else 1 (tiny debug shapes)
#define EW_VEC(T, cond, ...)                          \
  if (cond) { constexpr int VEC = 16 / sizeof(T); __VA_ARGS__; } \
  else { constexpr int VEC = 1; __VA_ARGS__; }

// row-per-workgroup kernels (4 16-B load groups in flight per lane) for the wide rows of the
// Llama MLPs; the grid-stride kernels otherwise (narrow / odd rows, debug shapes)
// act rows lda apart (lda > F: the act part of a K-augmented [act | s t] row)
void swiglu_fwd(DType dt, const void* gu, void* act, long N, int F, long lda, hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    EW_VEC(T, F % (16 / sizeof(T)) == 0 && lda % (16 / sizeof(T)) == 0, {
      if (F / VEC >= 512 && N <= 0x7fffffffL)
        hipLaunchKernelGGL((swiglu_fwd_rows_k<T, VEC, 4>), dim3((unsigned)N), dim3(256), 0, s, (const T*)gu,
                           (T*)act, F, lda);
      else
        hipLaunchKernelGGL((swiglu_fwd_k<T, VEC>), dim3(ew_grid(N * F / VEC)), dim3(256), 0, s, (const T*)gu,
                           (T*)act, N, F, lda);
    });
  });
}
bool swiglu_bwd_lr_ok(int r, int F) { return r == 16 && F % 8 == 0; }  // P slice: 128 VGPRs at r = 16
void swiglu_bwd_lr(DType dt, const void* gu, const void* base, long ldb, const void* u, long ldu, const void* P, int r,
                   float scale, void* dgu, long N, int F, hipStream_t s) {
  const dim3 grid((unsigned)((N + LR_ROWS - 1) / LR_ROWS));
#define LR_L(TT, RR) hipLaunchKernelGGL((swiglu_bwd_lr_k<TT, RR>), grid, dim3(256), 0, s, (const TT*)gu, (const TT*)base, \
                                        ldb, (const TT*)u, ldu, (const TT*)P, scale, (TT*)dgu, N, F)
  (void)r;
  if (dt == DType::BF16) LR_L(bf16_t, 16);
  else LR_L(f16_t, 16);
#undef LR_L
}
bool swiglu_bwd_lr_wgrad_ok(int r, int F) { return r == 16 && F % LRW_COLS == 0; }
int swiglu_bwd_lr_wgrad_splits(long N, int F) {
  // ~512 workgroups (two per CU at the kernel's register use), each row range >= 4 chunks
  const int slabs = F / LRW_COLS;
  int S = (512 + slabs - 1) / slabs;
  const long max_s = (N + 4 * LRW_CH - 1) / (4 * LRW_CH);
  if (S > max_s) S = (int)max_s;
  return S < 1 ? 1 : (S > 64 ? 64 : S);
}
void swiglu_bwd_lr_wgrad(DType dt, const void* gu, const void* base, long ldb, const void* u, long ldu, const void* P,
                         const void* st, long ldst, float scale, void* dgu, float* part, long N, int F, int S,
                         hipStream_t s) {
  const long rows_per = (N + S - 1) / S;
  const dim3 grid((unsigned)(F / LRW_COLS), (unsigned)S);
#define LRW_L(TT) hipLaunchKernelGGL((swiglu_bwd_lr_wg_k<TT>), grid, dim3(256), 0, s, (const TT*)gu, (const TT*)base, ldb, \
                                     (const TT*)u, ldu, (const TT*)P, (const TT*)st, ldst, scale, (TT*)dgu, part, N, F,   \
                                     rows_per)
  if (dt == DType::BF16) LRW_L(bf16_t);
  else LRW_L(f16_t);
#undef LRW_L
}
void swiglu_bwd(DType dt, const void* gu, const void* dact, void* dgu, void* act, long N, int F, hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    EW_VEC(T, F % (16 / sizeof(T)) == 0, {
      if (F / VEC >= 512 && N <= 0x7fffffffL)
        hipLaunchKernelGGL((swiglu_bwd_rows_k<T, VEC, 4>), dim3((unsigned)N), dim3(256), 0, s, (const T*)gu,
                           (const T*)dact, (T*)dgu, (T*)act, F);
      else
        hipLaunchKernelGGL((swiglu_bwd_k<T, VEC>), dim3(ew_grid(N * F / VEC)), dim3(256), 0, s, (const T*)gu,
                           (const T*)dact, (T*)dgu, (T*)act, N, F);
    });
  });
}
void gelu_fwd(DType dt, const void* f, void* g, long n, hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    EW_VEC(T, n % (16 / sizeof(T)) == 0, {
      hipLaunchKernelGGL((gelu_fwd_k<T, VEC>), dim3(ew_grid(n / VEC)), dim3(256), 0, s, (const T*)f, (T*)g,
                         n / VEC);
    });
  });
}
void gelu_bwd(DType dt, const void* f, const void* dg, void* df, long n, hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    EW_VEC(T, n % (16 / sizeof(T)) == 0, {
      hipLaunchKernelGGL((gelu_bwd_k<T, VEC>), dim3(ew_grid(n / VEC)), dim3(256), 0, s, (const T*)f,
                         (const T*)dg, (T*)df, n / VEC);
    });
  });
}
void dropout_add(DType dt, const void* x, const void* a, void* out, long n, float p, uint64_t seed,
                 uint64_t offset, hipStream_t s) {
  const uint32_t thr = drop_threshold16(p);
  const float inv_keep = drop_inv_keep(p);
  BLLM_DISPATCH(dt, T, {
    EW_VEC(T, n % (16 / sizeof(T)) == 0, {
      hipLaunchKernelGGL((dropout_add_k<T, VEC>), dim3(ew_grid(n / VEC)), dim3(256), 0, s, (const T*)x,
                         (const T*)a, (T*)out, n / VEC, seed, offset, thr, inv_keep);
    });
  });
}
void rope(DType dt, void* qkv, const float* cosT, const float* sinT, long N, int T_, int H, int G, int hd,
          bool inverse, int pos_offset, hipStream_t s, const int* pos_dev) {
  const int nh = H + G, stride = (H + 2 * G) * hd;
  const float sgn = inverse ? -1.f : 1.f;
  BLLM_DISPATCH(dt, T, {
    if constexpr (sizeof(T) == 2) {
      if ((hd / 2) % 8 == 0) {
        long tot = N * nh * (hd / 16);
        hipLaunchKernelGGL(rope_k<T>, dim3(ew_grid(tot)), dim3(256), 0, s, (T*)qkv, cosT, sinT, N, T_, nh, stride,
                           hd, pos_offset, sgn, pos_dev);
        return;
      }
    }
    {
      long tot = N * nh * (hd / 2);
      hipLaunchKernelGGL(rope_scalar_k<T>, dim3(ew_grid(tot)), dim3(256), 0, s, (T*)qkv, cosT, sinT, N, T_, nh,
                         stride, hd, pos_offset, sgn, pos_dev);
    }
  });
}

// ---------------------------------------------------------------- split-K partial sum
// out[e] (+)= sum_{s < S} part[s][e] in fp32, fixed order (deterministic); the reduction step
// of the split-K weight-gradient GEMMs (models/linear.py:_weight_grad).  8 elements per lane.
template <typename PT, typename OT>
__global__ __launch_bounds__(256) void sum_partials_k(const PT* __restrict__ part, OT* __restrict__ out, long n8,
                                                      int S, bool accumulate) {
  const long n = n8 * 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float acc[8];
    if (accumulate) {
      const VecN<OT, 8> o = ldv<OT, 8>(out + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = to_f(o.v[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    }
    for (int q = 0; q < S; ++q) {
      const VecN<PT, 8> p = ldv<PT, 8>(part + q * n + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += to_f(p.v[j]);
    }
    VecN<OT, 8> r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r.v[j] = from_f<OT>(acc[j]);
    stv<OT, 8>(out + i * 8, r);
  }
}

void sum_partials_into(DType pdt, DType odt, const void* part, void* out, long n, int S, bool accumulate,
                       hipStream_t s) {
  const long n8 = n / 8;
  BLLM_DISPATCH(pdt, PT, {
    BLLM_DISPATCH(odt, OT, {
      hipLaunchKernelGGL((sum_partials_k<PT, OT>), dim3(ew_grid(n8)), dim3(256), 0, s, (const PT*)part, (OT*)out,
                         n8, S, accumulate);
    });
  });
}

// ---------------------------------------------------------------- 2-D transpose (16-bit)
// out[C, R] = in[R, C]^T for bf16/fp16 (bit copy).  Used to give the input-gradient GEMM a
// K-contiguous weight (dX = dY W runs in hipBLASLt's fast "both operands K-contiguous" layout).
// 64x64 tile per workgroup through LDS: 16-byte row loads, LDS row stride 66 halves (33 dwords)
// so the column gathers of one wave land on distinct banks, 16-byte row stores.
constexpr int TP_T = 64, TP_LD = TP_T + 2;
__global__ __launch_bounds__(256) void transpose16_k(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                     long R, long C) {
  __shared__ uint16_t tile[TP_T * TP_LD];
  const long ntc = (C + TP_T - 1) / TP_T;
  const long r0 = (long)(blockIdx.x / ntc) * TP_T, c0 = (long)(blockIdx.x % ntc) * TP_T;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = t + k * 256, row = v >> 3, cv = (v & 7) * 8;
    uint4 x = make_uint4(0, 0, 0, 0);
    if (r0 + row < R && c0 + cv < C) x = *reinterpret_cast<const uint4*>(in + (r0 + row) * C + c0 + cv);
    uint32_t* d = reinterpret_cast<uint32_t*>(tile + row * TP_LD + cv);
    d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int ov = (t & 7) * 8, orow = (t >> 3) + k * 32;
    if (c0 + orow >= C || r0 + ov >= R) continue;
    uint16_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = tile[(ov + j) * TP_LD + orow];
    uint4 y;
    y.x = e[0] | ((uint32_t)e[1] << 16); y.y = e[2] | ((uint32_t)e[3] << 16);
    y.z = e[4] | ((uint32_t)e[5] << 16); y.w = e[6] | ((uint32_t)e[7] << 16);
    *reinterpret_cast<uint4*>(out + (c0 + orow) * R + r0 + ov) = y;
  }
}

void transpose16(const void* in, void* out, long R, long C, hipStream_t s) {
  const long nt = ((R + TP_T - 1) / TP_T) * ((C + TP_T - 1) / TP_T);
  hipLaunchKernelGGL(transpose16_k, dim3((unsigned)nt), dim3(256), 0, s, (const uint16_t*)in, (uint16_t*)out, R, C);
}

}  // namespace bllm
