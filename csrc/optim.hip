// Fused AdamW over flat parameter buffers + multi-tensor squared L2 norm.
//
// Replaces torch.optim.AdamW(lr, weight_decay=0.1) (reference build_components.py:250-258)
// and clip_grad_norm_(max_norm=1.0) (train.py:114-120).  One launch per flat unit buffer:
// reads grad (bf16/f16/f32) + fp32 master/exp_avg/exp_avg_sq, writes them back plus the
// low-precision param copy — 16-B vector accesses, pure HBM streaming.  The clip factor
// (and the fp16 loss-scale inverse) arrive as a DEVICE scalar, so clipping never forces a
// host sync.  The norm is two-level and order-fixed (deterministic).
#include "common.h"

namespace bllm {

// UNROLL independent VEC-groups per thread per iteration keep more loads in flight (the
// kernel streams 28 B/param once: every access is a non-temporal load/store so the stream
// does not evict L2/MALL-resident data of the overlapped forward).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <typename T, int N>
__device__ __forceinline__ VecN<T, N> ldnt(const T* p) {
  VecN<T, N> r;
  if constexpr (sizeof(r) == 16) {
    const u32x4 u = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    __builtin_memcpy(&r, &u, 16);
  } else if constexpr (sizeof(r) == 8) {
    const u32x2 u = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    __builtin_memcpy(&r, &u, 8);
  } else {
    r = ldv<T, N>(p);
  }
  return r;
}
template <typename T, int N>
__device__ __forceinline__ void stnt(T* p, const VecN<T, N>& r) {
  if constexpr (sizeof(r) == 16) {
    u32x4 u;
    __builtin_memcpy(&u, &r, 16);
    __builtin_nontemporal_store(u, reinterpret_cast<u32x4*>(p));
  } else if constexpr (sizeof(r) == 8) {
    u32x2 u;
    __builtin_memcpy(&u, &r, 8);
    __builtin_nontemporal_store(u, reinterpret_cast<u32x2*>(p));
  } else {
    stv<T, N>(p, r);
  }
}

template <typename P, typename G, int VEC, int UNROLL>
__global__ __launch_bounds__(256) void adamw_k(P* __restrict__ param, float* __restrict__ master,
                                               const G* __restrict__ grad, float* __restrict__ m,
                                               float* __restrict__ v, long nvec, float lr, float b1, float b2,
                                               float eps, float wd, float bc1, float bc2_sqrt,
                                               const float* __restrict__ gscale) {
  const float gs = gscale ? gscale[0] : 1.f;
  const float decay = 1.f - lr * wd;
  const float step = lr / bc1;
  const long stride = (long)gridDim.x * 256 * UNROLL;
  for (long i0 = blockIdx.x * 256L * UNROLL + threadIdx.x; i0 < nvec; i0 += stride) {
    VecN<G, VEC> gv[UNROLL];
    VecN<float, VEC> mv[UNROLL], vv[UNROLL], pv[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const long i = i0 + u * 256L;
      if (i < nvec) {
        const long o = i * VEC;
        gv[u] = ldnt<G, VEC>(grad + o);
        mv[u] = ldnt<float, VEC>(m + o);
        vv[u] = ldnt<float, VEC>(v + o);
        if (master) pv[u] = ldnt<float, VEC>(master + o);
        else {
          VecN<P, VEC> pp = ldv<P, VEC>(param + o);
#pragma unroll
          for (int j = 0; j < VEC; ++j) pv[u].v[j] = to_f(pp.v[j]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const long i = i0 + u * 256L;
      if (i < nvec) {
        const long o = i * VEC;
        VecN<P, VEC> po;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float g = to_f(gv[u].v[j]) * gs;
          mv[u].v[j] = b1 * mv[u].v[j] + (1.f - b1) * g;
          vv[u].v[j] = b2 * vv[u].v[j] + (1.f - b2) * g * g;
          float p = pv[u].v[j] * decay;
          p -= step * mv[u].v[j] / (sqrtf(vv[u].v[j]) / bc2_sqrt + eps);
          pv[u].v[j] = p;
          po.v[j] = from_f<P>(p);
        }
        stnt<float, VEC>(m + o, mv[u]);
        stnt<float, VEC>(v + o, vv[u]);
        if (master) stnt<float, VEC>(master + o, pv[u]);
        stnt<P, VEC>(param + o, po);
      }
    }
  }
}

// 4 independent 16-B loads per thread per iteration (4 accumulators) keep enough bytes in
// flight per CU to stream at HBM rate; the partials are summed in a fixed order (sum_k).
template <typename T, int VEC>
__global__ __launch_bounds__(256) void sqsum_partial_k(const T* __restrict__ x, long nvec, float* __restrict__ part) {
  __shared__ float red[4];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + 3 * stride < nvec; i += 4 * stride) {
    const VecN<T, VEC> a = ldv<T, VEC>(x + i * VEC), b = ldv<T, VEC>(x + (i + stride) * VEC);
    const VecN<T, VEC> c = ldv<T, VEC>(x + (i + 2 * stride) * VEC), d = ldv<T, VEC>(x + (i + 3 * stride) * VEC);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float f = to_f(a.v[j]); s0 += f * f;
      f = to_f(b.v[j]); s1 += f * f;
      f = to_f(c.v[j]); s2 += f * f;
      f = to_f(d.v[j]); s3 += f * f;
    }
  }
  for (; i < nvec; i += stride) {
    const VecN<T, VEC> a = ldv<T, VEC>(x + i * VEC);
#pragma unroll
    for (int j = 0; j < VEC; ++j) { const float f = to_f(a.v[j]); s0 += f * f; }
  }
  float s = (s0 + s1) + (s2 + s3);
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void sum_k(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) out[0] = s;
}

template <typename P, typename G>
static void adamw_launch(void* param, float* master, const void* grad, float* m, float* v, long n, float lr,
                         float b1, float b2, float eps, float wd, float bc1, float bc2s, const float* gscale,
                         hipStream_t s) {
  if (n % 4 == 0) {
    long nv = n / 4;
    int g = (int)((nv + 511) / 512 < 2048 ? (nv + 511) / 512 : 2048);
    hipLaunchKernelGGL((adamw_k<P, G, 4, 2>), dim3(g > 0 ? g : 1), dim3(256), 0, s, (P*)param, master,
                       (const G*)grad, m, v, nv, lr, b1, b2, eps, wd, bc1, bc2s, gscale);
  } else {
    int g = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL((adamw_k<P, G, 1, 1>), dim3(g > 0 ? g : 1), dim3(256), 0, s, (P*)param, master,
                       (const G*)grad, m, v, n, lr, b1, b2, eps, wd, bc1, bc2s, gscale);
  }
}

void adamw_step(DType pdt, DType gdt, void* param, float* master, const void* grad, float* m, float* v, long n,
                float lr, float b1, float b2, float eps, float wd, int step, const float* gscale, hipStream_t s) {
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2s = sqrtf(1.f - powf(b2, (float)step));
  BLLM_DISPATCH(pdt, P, {
    BLLM_DISPATCH(gdt, G, (adamw_launch<P, G>(param, master, grad, m, v, n, lr, b1, b2, eps, wd, bc1, bc2s,
                                              gscale, s)));
  });
}

// number of partial slots the launcher will use for a tensor of n elements
int sqsum_slots(long n) {
  long g = (n + 256L * 32 - 1) / (256L * 32);
  return (int)(g < 1024 ? (g > 0 ? g : 1) : 1024);
}

void sqsum_partial(DType dt, const void* x, long n, float* part, int slots, hipStream_t s) {
  BLLM_DISPATCH(dt, T, {
    if (n % (16 / sizeof(T)) == 0) {
      constexpr int VEC = 16 / sizeof(T);
      hipLaunchKernelGGL((sqsum_partial_k<T, VEC>), dim3(slots), dim3(256), 0, s, (const T*)x, n / VEC, part);
    } else {
      hipLaunchKernelGGL((sqsum_partial_k<T, 1>), dim3(slots), dim3(256), 0, s, (const T*)x, n, part);
    }
  });
}

void sum_partials(const float* part, int n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(sum_k, dim3(1), dim3(256), 0, s, part, n, out);
}

}  // namespace bllm
