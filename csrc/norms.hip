#include <stdlib.h>
// RMSNorm / LayerNorm forward + backward (fused residual-gradient add) for gfx950.
//
// Replaces reference Models/Llama/common_components.py:54-70 (RMSNorm) and nn.LayerNorm
// (Models/GPT2/GPT2.py:79-80).  Memory-bound: one wave64 per row, the row held in VGPRs
// (16-B loads, NV vectors per lane), fp32 statistics, one pass over x in forward and one
// over (x, dy[, dx_acc]) in backward (one workgroup per row there).  Weight/bias gradients:
// per-thread register accumulators for the columns a thread owns -> one fp32 partial row per
// workgroup -> a column-reduction kernel (deterministic, no global atomics).
#include <cstdlib>
#include "common.h"

namespace bllm {

constexpr int ROWS_PER_WG = 4;  // 4 waves x 1 row
// backward workgroups (rows are grid-strided over them): 1024 = 4 WGs / 16 waves per CU on 256 CUs,
// enough loads in flight for a d=4096 row pass; each WG adds one fp32 dW partial row (16 MiB at
// d=4096), which col_reduce_k streams once
constexpr int MAX_BWD_WG = 1024;

// Residual-dropout prologue (ADD, GPT-2's attention residual + norm2 in one pass):
//   xs = x + dropout(a) is stored (rounded to T) and normalised, bitwise dropout_add_k then
//   norm_fwd_k (same keep bits at element index row * d + column, same lane -> column map).
struct AddDrop {
  const void* a = nullptr;
  void* xs = nullptr;
  uint64_t seed = 0, offset = 0;
  uint32_t thr = 0;
  float inv_keep = 1.f;
};

template <typename T, int NV, bool LN, bool ADD = false>
__global__ __launch_bounds__(256) void norm_fwd_k(const T* __restrict__ x, const T* __restrict__ w,
                                                  const T* __restrict__ b, T* __restrict__ y,
                                                  float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                  int N, int d, float eps, long ldy, AddDrop ad = AddDrop{}) {
  // no FMA contraction: every instantiation (ADD or not) rounds identically, so the fused
  // residual + norm pass is bitwise the two separate kernels
#pragma clang fp contract(off)
  constexpr int VEC = 16 / sizeof(T);
  const int row = blockIdx.x * ROWS_PER_WG + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const int nvec = d / VEC;
  const T* xr = x + (size_t)row * d;
  float v[NV][VEC];
  float s1 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nvec) {
      Vec16<T> r = ld16(xr + c * VEC);
      if constexpr (ADD) {
        const Vec16<T> av = ld16(static_cast<const T*>(ad.a) + (size_t)row * d + c * VEC);
        uint32_t bits[VEC];
        drop_bits_run<VEC>(ad.seed, ad.offset + (uint64_t)row * d + c * VEC, bits);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          float t = bits[j] >= ad.thr ? to_f(av.v[j]) * ad.inv_keep : 0.f;
          t += to_f(r.v[j]);
          r.v[j] = from_f<T>(t);
        }
        st16(static_cast<T*>(ad.xs) + (size_t)row * d + c * VEC, r);
      }
#pragma unroll
      for (int j = 0; j < VEC; ++j) { v[i][j] = to_f(r.v[j]); s1 += LN ? v[i][j] : v[i][j] * v[i][j]; }
    }
  }
  s1 = wave_sum(s1);
  float mu = 0.f, rs;
  if (LN) {
    mu = s1 / d;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      if (c < nvec) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) { float t = v[i][j] - mu; s2 += t * t; }
      }
    }
    s2 = wave_sum(s2);
    rs = rsqrtf(s2 / d + eps);
  } else {
    rs = rsqrtf(s1 / d + eps);
  }
  T* yr = y + (size_t)row * ldy;  // ldy > d: written into the x part of a K-augmented [x | s t] row
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < nvec) {
      Vec16<T> wv = ld16(w + c * VEC), o;
      if (LN) {
        Vec16<T> bv = ld16(b + c * VEC);
#pragma unroll
        for (int j = 0; j < VEC; ++j) o.v[j] = from_f<T>((v[i][j] - mu) * rs * to_f(wv.v[j]) + to_f(bv.v[j]));
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) o.v[j] = from_f<T>(v[i][j] * rs * to_f(wv.v[j]));
      }
      st16(yr + c * VEC, o);
    }
  }
  if (lane == 0) {
    rstd_out[row] = rs;
    if (LN) mean_out[row] = mu;
  }
}

// backward: dx = rs * (g - [LN: mean(g)] - xhat * mean(g * xhat)) (+ dx_acc), g = dy * w
// One WORKGROUP per row (rows grid-strided): a row of d=4096 bf16 is 512 16-B vectors, i.e.
// NV=2 per thread at 256 threads, so the per-thread state (raw x/dy vectors + the dW/dB
// column accumulators, which each thread owns exclusively for its columns) stays far below
// the VGPR budget and several workgroups share a CU to hide HBM latency.  The two row sums
// cross the 4 waves through a parity-double-buffered LDS slot (one barrier per row).  Each
// workgroup writes one fp32 partial row for dW (and dB); col_reduce_k sums them in a fixed
// order (deterministic, no global atomics).
template <typename T, int NV, bool LN, bool PF>
__global__ __launch_bounds__(256) void norm_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                  const T* __restrict__ w, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, const T* __restrict__ dx_acc,
                                                  T* __restrict__ dx, float* __restrict__ part_w,
                                                  float* __restrict__ part_b, int N, int d) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float red[2][4][2];
  const int tid = threadIdx.x, lane = tid & 63, wv_id = tid >> 6;
  const int nwaves = blockDim.x >> 6;
  const int nvec = d / VEC;
  float aw[NV][VEC], ab[LN ? NV : 1][VEC];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      aw[i][j] = 0.f;
      if (LN) ab[LN ? i : 0][j] = 0.f;
    }
  // PF (rows shorter than 4 waves): the next row's x / dy / dx_acc are loaded before this row is
  // reduced (register double buffer) -- with one row in flight per workgroup a GPT-2 row
  // (d = 1280, 3 waves) kept too few loads outstanding: 170 -> 149 us per call (3.9 -> 4.5 TB/s).
  // At d = 4096 the same prefetch measured 256 -> 284 us, so 4-wave rows keep the single-row
  // form (profiles/r6/normpf/).  w is loaded once per workgroup.
  Vec16<T> wv[NV], xv[NV], dv[NV], av[NV], nx[NV], nd[NV], na[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + (int)blockDim.x * i;
    if (c < nvec) wv[i] = ld16(w + c * VEC);
  }
  auto load_row = [&](int r, Vec16<T> (&lx)[NV], Vec16<T> (&ld)[NV], Vec16<T> (&la)[NV]) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = tid + (int)blockDim.x * i;
      if (c < nvec) {
        lx[i] = ld16(x + (size_t)r * d + c * VEC);
        ld[i] = ld16(dy + (size_t)r * d + c * VEC);
        if (dx_acc) la[i] = ld16(dx_acc + (size_t)r * d + c * VEC);
      }
    }
  };
  int par = 0;
  if constexpr (PF) {
    if ((int)blockIdx.x < N) load_row(blockIdx.x, xv, dv, av);
  }
  for (int row = blockIdx.x; row < N; row += gridDim.x, par ^= 1) {
    if constexpr (PF) {
      const int rn = row + (int)gridDim.x;
      if (rn < N) load_row(rn, nx, nd, na);
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = tid + (int)blockDim.x * i;
        if (c < nvec) {
          xv[i] = ld16(x + (size_t)row * d + c * VEC);
          dv[i] = ld16(dy + (size_t)row * d + c * VEC);
        }
      }
    }
    const float rs = rstd[row];
    const float mu = LN ? mean[row] : 0.f;
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = tid + (int)blockDim.x * i;
      if (c < nvec) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float dd = to_f(dv[i].v[j]);
          const float xh = (to_f(xv[i].v[j]) - mu) * rs;
          const float gg = dd * to_f(wv[i].v[j]);
          aw[i][j] += dd * xh;
          if (LN) ab[LN ? i : 0][j] += dd;
          sg += gg;
          sgx += gg * xh;
        }
      }
    }
    sgx = wave_sum(sgx);
    if (LN) sg = wave_sum(sg);
    if (lane == 0) {
      red[par][wv_id][0] = sgx;
      red[par][wv_id][1] = sg;
    }
    __syncthreads();
    sgx = 0.f;
    sg = 0.f;
    for (int k = 0; k < nwaves; ++k) {
      sgx += red[par][k][0];
      if (LN) sg += red[par][k][1];
    }
    sgx /= d;
    sg /= d;
    T* dxr = dx + (size_t)row * d;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = tid + (int)blockDim.x * i;
      if (c < nvec) {
        Vec16<T> o;
        if (!PF && dx_acc) av[i] = ld16(dx_acc + (size_t)row * d + c * VEC);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float xh = (to_f(xv[i].v[j]) - mu) * rs;
          const float gg = to_f(dv[i].v[j]) * to_f(wv[i].v[j]);
          float r = rs * (gg - (LN ? sg : 0.f) - xh * sgx);
          if (dx_acc) r += to_f(av[i].v[j]);
          o.v[j] = from_f<T>(r);
        }
        st16(dxr + c * VEC, o);
      }
    }
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        xv[i] = nx[i];
        dv[i] = nd[i];
        if (dx_acc) av[i] = na[i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = tid + (int)blockDim.x * i;
    if (c < nvec) {
      float* pw = part_w + (size_t)blockIdx.x * d + c * VEC;
#pragma unroll
      for (int j = 0; j < VEC; j += 4)
        *reinterpret_cast<float4*>(pw + j) = make_float4(aw[i][j], aw[i][j + 1], aw[i][j + 2], aw[i][j + 3]);
      if (LN) {
        float* pb = part_b + (size_t)blockIdx.x * d + c * VEC;
#pragma unroll
        for (int j = 0; j < VEC; j += 4)
          *reinterpret_cast<float4*>(pb + j) = make_float4(ab[LN ? i : 0][j], ab[LN ? i : 0][j + 1],
                                                           ab[LN ? i : 0][j + 2], ab[LN ? i : 0][j + 3]);
      }
    }
  }
}

template <typename OT>
__global__ __launch_bounds__(256) void col_reduce_k(const float* __restrict__ part, OT* __restrict__ out, int P,
                                                    int d, bool accumulate) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float s = 0.f, s2 = 0.f;
  if (c < d) {
    int p = g;
#pragma unroll 4
    for (; p + 16 < P; p += 32) {  // two independent chains keep more loads in flight
      s += part[(size_t)p * d + c];
      s2 += part[(size_t)(p + 16) * d + c];
    }
    if (p < P) s += part[(size_t)p * d + c];
  }
  red[g][cl] = s + s2;
  __syncthreads();
  if (threadIdx.x < 16 && c < d) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    if (accumulate) t += to_f(out[c]);
    out[c] = from_f<OT>(t);
  }
}

// sum P fp32 partial rows into out[d] (dtype odt; written or accumulated) in a fixed order
void col_reduce(const float* part, DType odt, void* out, int P, int d, bool accumulate, hipStream_t s) {
  BLLM_DISPATCH(odt, OT, {
    hipLaunchKernelGGL(col_reduce_k<OT>, dim3(ceil_div(d, 16)), dim3(256), 0, s, part, (OT*)out, P, d, accumulate);
  });
}

// ----------------------------------------------------------------------------- launchers
template <typename T, bool LN, bool ADD = false>
static void fwd_dispatch(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                         int N, int d, float eps, long ldy, hipStream_t s, AddDrop ad = AddDrop{}) {
  constexpr int VEC = 16 / sizeof(T);
  const int nvec = d / VEC;
  const int nv = (nvec + 63) / 64;
  dim3 grid(ceil_div(N, ROWS_PER_WG)), block(256);
#define L(NVV) hipLaunchKernelGGL((norm_fwd_k<T, NVV, LN, ADD>), grid, block, 0, s, (const T*)x, (const T*)w, \
                                  (const T*)b, (T*)y, mean, rstd, N, d, eps, ldy, ad)
  if (nv <= 1) L(1); else if (nv <= 2) L(2); else if (nv <= 4) L(4); else if (nv <= 8) L(8); else L(16);
#undef L
}

template <typename T, bool LN>
static void bwd_dispatch(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                         const void* dx_acc, void* dx, float* part_w, float* part_b, DType odt, void* dw, void* db,
                         bool accumulate, int N, int d, int nwg, hipStream_t s) {
  constexpr int VEC = 16 / sizeof(T);
  const int nvec = d / VEC;
  // threads per row: a multiple of 64 covering the row in <= 4 waves; NV vectors per thread
  const int bt = nvec >= 256 ? 256 : ceil_div(nvec, 64) * 64;
  const int nv = ceil_div(nvec, bt);
  dim3 grid(nwg), block(bt);
#define L(NVV, PF) hipLaunchKernelGGL((norm_bwd_k<T, NVV, LN, PF>), grid, block, 0, s, (const T*)dy, (const T*)x, \
                                      (const T*)w, mean, rstd, (const T*)dx_acc, (T*)dx, part_w, part_b, N, d)
  if (bt < 256) L(1, true); else if (nv <= 1) L(1, false); else if (nv <= 2) L(2, false); else L(4, false);
#undef L
  col_reduce(part_w, odt, dw, nwg, d, accumulate, s);
  if (LN) col_reduce(part_b, odt, db, nwg, d, accumulate, s);
}

// partial rows of the dW / dB sums = backward workgroups
int norm_bwd_num_wg(int N, int d) {
  (void)d;
  return N < MAX_BWD_WG ? N : MAX_BWD_WG;
}

// max supported row length per dtype (NV <= 16): 8192 (bf16/f16), 4096 (f32)
int norm_max_dim(DType dt) { return dt == DType::F32 ? 4096 : 8192; }

void rmsnorm_fwd(DType dt, const void* x, const void* w, void* y, float* rstd, int N, int d, float eps, long ldy,
                 hipStream_t s) {
  BLLM_DISPATCH(dt, T, (fwd_dispatch<T, false>(x, w, nullptr, y, nullptr, rstd, N, d, eps, ldy, s)));
}
void layernorm_fwd(DType dt, const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                   int N, int d, float eps, hipStream_t s) {
  BLLM_DISPATCH(dt, T, (fwd_dispatch<T, true>(x, w, b, y, mean, rstd, N, d, eps, (long)d, s)));
}
void rmsnorm_bwd(DType dt, const void* dy, const void* x, const void* w, const float* rstd, const void* dx_acc,
                 void* dx, float* part, DType odt, void* dw, bool accumulate, int N, int d, int nwg, hipStream_t s) {
  BLLM_DISPATCH(dt, T, (bwd_dispatch<T, false>(dy, x, w, nullptr, rstd, dx_acc, dx, part, nullptr, odt, dw,
                                               nullptr, accumulate, N, d, nwg, s)));
}
void layernorm_bwd(DType dt, const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                   const void* dx_acc, void* dx, float* part_w, float* part_b, DType odt, void* dw, void* db,
                   bool accumulate, int N, int d, int nwg, hipStream_t s) {
  BLLM_DISPATCH(dt, T, (bwd_dispatch<T, true>(dy, x, w, mean, rstd, dx_acc, dx, part_w, part_b, odt, dw, db,
                                              accumulate, N, d, nwg, s)));
}

void dropout_add_layernorm_fwd(DType dt, const void* x, const void* a, void* xs, const void* w, const void* b, void* y,
                               float* mean, float* rstd, int N, int d, float eps, float p, uint64_t seed,
                               uint64_t offset, hipStream_t s) {
  AddDrop ad;
  ad.a = a;
  ad.xs = xs;
  ad.seed = seed;
  ad.offset = offset;
  ad.thr = drop_threshold16(p);
  ad.inv_keep = drop_inv_keep(p);
  BLLM_DISPATCH(dt, T, (fwd_dispatch<T, true, true>(x, w, b, y, mean, rstd, N, d, eps, (long)d, s, ad)));
}

}  // namespace bllm
