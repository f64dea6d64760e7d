// Shared device helpers for the gfx950 (CDNA4, MI355X) kernel library.
//
// Conventions used by every kernel in csrc/:
//  * wave64: all cross-lane reductions are over 64 lanes (__shfl_xor 32..1);
//  * memory-bound kernels move 16 bytes per lane per access (8 x bf16/fp16, 4 x fp32),
//    per the CDNA guide's "vectorize always" rule (scalar bf16 loads cost ~2x);
//  * all math in fp32; storage type T in {float, __bf16, _Float16};
//  * the dropout RNG is a stateless counter hash so masks are regenerated (never stored)
//    in backward and in activation-checkpoint recompute — bit-identical to
//    ops/reference.py::drop_keep_mask.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bllm {

enum class DType : int { F32 = 0, BF16 = 1, F16 = 2 };

typedef __bf16 bf16_t;
typedef _Float16 f16_t;

template <typename T> __device__ __forceinline__ float to_f(T x) { return static_cast<float>(x); }
template <typename T> __device__ __forceinline__ T from_f(float x) { return static_cast<T>(x); }

// 16-byte vector of T
template <typename T> struct Vec16 {
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};

template <typename T>
__device__ __forceinline__ Vec16<T> ld16(const T* p) {
  Vec16<T> r;
  *reinterpret_cast<uint4*>(&r) = *reinterpret_cast<const uint4*>(p);
  return r;
}
template <typename T>
__device__ __forceinline__ void st16(T* p, const Vec16<T>& r) {
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(&r);
}

// N-element vector of T (N*sizeof(T) bytes, naturally aligned loads when possible)
template <typename T, int N> struct VecN { T v[N]; };
// callers guarantee natural alignment of the whole vector (sizes are multiples of N)
template <typename T, int N>
__device__ __forceinline__ VecN<T, N> ldv(const T* p) {
  VecN<T, N> r;
  if constexpr (sizeof(r) == 16) *reinterpret_cast<uint4*>(&r) = *reinterpret_cast<const uint4*>(p);
  else if constexpr (sizeof(r) == 8) *reinterpret_cast<uint2*>(&r) = *reinterpret_cast<const uint2*>(p);
  else {
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = p[i];
  }
  return r;
}
template <typename T, int N>
__device__ __forceinline__ void stv(T* p, const VecN<T, N>& r) {
  if constexpr (sizeof(r) == 16) *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(&r);
  else if constexpr (sizeof(r) == 8) *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(&r);
  else {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = r.v[i];
  }
}

// SiLU gate sigma(a) = 1 / (1 + e^-a) on v_rcp_f32 (1 ulp): the IEEE division sequence (~10 VALU
// instructions, two per element) made the SwiGLU passes VALU-bound.  Every SwiGLU kernel and the
// GEMM epilogue form act = (a * sigma) * up from this one helper, so act is bitwise the same
// wherever it is (re)computed.
__device__ __forceinline__ float silu_sig(float a) { return __builtin_amdgcn_rcpf(1.f + __expf(-a)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x == NT (multiple of 64); red must hold NT/64 floats
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

// ---------------------------------------------------------------- GELU derivative
// d/dx [x Phi(x)] = Phi(x) + x phi(x) for the exact (erf) GELU, branch-free: Phi from
// Abramowitz-Stegun 7.1.26 (|erf error| <= 1.5e-7, about one fp32 ulp of Phi) sharing its
// exp(-x^2 / 2) with phi.  libm's erff branches by range (divergent in a wave) and made the GELU
// backward passes VALU-bound (~100 instructions per element); this is ~15, all full-rate but one
// v_exp and one v_rcp.
// Phi(x) (standard normal CDF) and phi(x) on the A&S 7.1.26 erfc form (abs. error 1.5e-7):
// branch-free, ~15 full-rate instructions
__device__ __forceinline__ float norm_cdf_pdf(float x, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  // v_rcp_f32 (1 ulp): __frcp_rn lowers to the IEEE division sequence (div_scale / div_fmas /
  // div_fixup, ~10 instructions), more than the rest of the function; A&S 7.1.26 is 1.5e-7 anyway
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * z);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float e = __expf(-0.5f * x * x);
  const float tail = 0.5f * poly * e;                  // 1 - Phi(|x|)
  pdf = e * 0.39894228040143268f;
  return x >= 0.f ? 1.f - tail : tail;
}
__device__ __forceinline__ float gelu_grad(float x) {
  float pdf;
  const float cdf = norm_cdf_pdf(x, pdf);
  return cdf + x * pdf;
}
// exact-erf GELU x Phi(x).  16-bit outputs use the A&S form above (its 1.5e-7 is far below a
// bf16 / fp16 rounding unit, and libm's range-branching erff cost ~100 VALU instructions per
// element -- the reason the fused c_fc + bias + GELU GEMM epilogue lost to the separate pass);
// fp32 keeps libm's erff.  Every GELU forward (the elementwise kernel, the GEMM epilogue and the
// GELU backward's rebuild of g) goes through this one function, so g is bitwise the same
// wherever it is (re)computed.
template <typename T> __device__ __forceinline__ float gelu_fwd_f(float x) {
  if constexpr (sizeof(T) == 2) {
    float pdf;
    return x * norm_cdf_pdf(x, pdf);
  } else {
    return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  }
}

// ---------------------------------------------------------------- dropout RNG
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// Counter-based dropout: ONE 32-bit hash per PAIR of consecutive element indices, 16 bits per
// element; keep iff bits >= thr16 = floor(p * 2^16) (p resolution 1.5e-5).  Every kernel and the
// CPU oracle (ops/reference.py:drop_keep_mask) use exactly this function of (seed, index).
__device__ __forceinline__ uint32_t drop_seed_mix(uint64_t seed, uint32_t pair_hi) {
  return mix32((uint32_t)seed + pair_hi * 0x9E3779B9u);
}
__device__ __forceinline__ uint32_t drop_pair(uint64_t seed, uint64_t pair) {
  return mix32((uint32_t)pair ^ drop_seed_mix(seed, (uint32_t)(pair >> 32)));
}
__device__ __forceinline__ uint32_t drop_bits16(uint64_t seed, uint64_t idx) {
  const uint32_t h = drop_pair(seed, idx >> 1);
  return (idx & 1) ? (h >> 16) : (h & 0xFFFFu);
}
// Dropout bits inside one attention (batch, head) slab [base, base + T*T) (T <= 65536, so the
// slab spans at most two 2^32-pair windows): the seed mix of both windows is computed once and
// each pair then costs a single mix32.
struct DropSlab {
  uint32_t sm0, sm1, hi0;
  __device__ __forceinline__ void init(uint64_t seed, uint64_t base) {
    hi0 = (uint32_t)(base >> 33);
    sm0 = drop_seed_mix(seed, hi0);
    sm1 = drop_seed_mix(seed, hi0 + 1);
  }
  __device__ __forceinline__ uint32_t pair_hash(uint64_t pair) const {
    return mix32((uint32_t)pair ^ ((uint32_t)(pair >> 32) == hi0 ? sm0 : sm1));
  }
  __device__ __forceinline__ uint32_t bits16(uint64_t idx) const {
    const uint32_t h = pair_hash(idx >> 1);
    return (idx & 1) ? (h >> 16) : (h & 0xFFFFu);
  }
};
// bits of VEC consecutive indices from e0; pairs share one hash when e0 is even
template <int VEC>
__device__ __forceinline__ void drop_bits_run(uint64_t seed, uint64_t e0, uint32_t (&bits)[VEC]) {
  if ((e0 & 1) == 0) {
#pragma unroll
    for (int j = 0; j < VEC; j += 2) {
      const uint32_t h = drop_pair(seed, (e0 + j) >> 1);
      bits[j] = h & 0xFFFFu;
      if (j + 1 < VEC) bits[j + 1] = h >> 16;
    }
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) bits[j] = drop_bits16(seed, e0 + j);
  }
}
inline uint32_t drop_threshold16(float p) {
  const double t = (double)p * 65536.0;
  return t >= 65536.0 ? 65536u : (uint32_t)t;
}
// exact inverse of the realised keep probability (1 - thr16 / 2^16)
inline float drop_inv_keep(float p) {
  const uint32_t t = drop_threshold16(p);
  return t >= 65536u ? 0.f : (float)(65536.0 / (65536.0 - (double)t));
}

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4) issued from inline asm so hipcc does
// not track it: the compiler otherwise guards every later ds_read with s_waitcnt vmcnt(0)
// (it cannot prove the in-flight DMA targets the other LDS buffer), which serialises the
// prefetch with compute.  The caller drains it with an explicit vmcnt before the barrier that
// precedes the reads (cdna_hip_programming.md §5.7).  ``lds_dst`` is the wave-uniform base;
// lane i writes lds_dst + 16*i.
__device__ __forceinline__ void glds16(const void* gsrc, const void* lds_dst) {
  uint32_t lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst;
  lds = __builtin_amdgcn_readfirstlane(lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, const void* lds_dst) {
  uint32_t lds = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst;
  lds = __builtin_amdgcn_readfirstlane(lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// wait until at most N vector-memory ops of this wave are outstanding (prefetch depth > 1)
template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// wave-uniform 64-bit pointer materialised in SGPRs (for the saddr form of LDS-DMA)
__device__ __forceinline__ const void* sgpr_ptr(const void* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p);
}
// LDS-DMA, saddr form: uniform SGPR base + per-lane 32-bit byte offset (loop-invariant, so a
// tile step needs no per-lane address arithmetic); lds_dst is a wave-uniform LDS byte address.
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_dst) : "memory");
}

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Workgroup order of the attention kernels: a grid of nblk blocks (query or key blocks, heaviest
// first) x nunit units ((batch, head) or (batch, kv head)); units come in groups of gsz that read
// one K/V stream (the query heads of a kv head).  Workgroup lin runs on XCD lin % 8 (round-robin
// dispatch).
//   xmap 0: block-major over all units (unit = lin % nunit);
//   xmap 1: XCD x owns the groups with index % 8 == x and runs them block-major, the units of a
//           group back to back: the query heads that share a K/V stream read it through one L2
//           (nunit / gsz must be a multiple of 8, attn_xcd_order_ok).  Round 6: Llama-3-8B B=40
//           forward 658 -> 730 TF/s, Llama-3.2-1B 624 -> 675, backward 1.717 -> 1.660 ms (the dQ
//           kernel; its K/V streams are shared the same way), MHA (GPT-2) unchanged
//           (profiles/r6/attn/xcd/).  Measured and dropped: group-major order (each group's
//           blocks back to back), worse on three of four forward shapes and, for the dK/dV grid
//           alone, on all five backward shapes (+5-17 %, profiles/r6/attn/xcd/kv_order.jsonl).
__device__ __forceinline__ void attn_wg_order(int lin, int nunit, int gsz, int xmap, int& blk, int& unit) {
  if (xmap == 0) {
    blk = lin / nunit;
    unit = lin - blk * nunit;
    return;
  }
  const int x = lin & 7, k = lin >> 3;
  const int per_blk = (nunit / gsz / 8) * gsz;
  blk = k / per_blk;
  const int rem = k - blk * per_blk, gl = rem / gsz;
  unit = (gl * 8 + x) * gsz + (rem - gl * gsz);
}
inline bool attn_xcd_order_ok(int nunit, int gsz) { return gsz > 0 && nunit % gsz == 0 && (nunit / gsz) % 8 == 0; }

// ---- kernel debug mode (tools/build_ext.py --debug -> _C_debug.so, loaded when
// BLLM_KERNEL_DEBUG=1).  BLLM_DASSERT records the first failed check of a translation unit in a
// device word with a vector atomic and lets the kernel run on (no trap: a fault would take the
// whole device down); ops/__init__.py synchronises after every op in debug mode and raises with
// the check's name (bllm::debug_error).  Release builds compile every check away.
enum DebugCode : unsigned int {
  DBG_OK = 0,
  DBG_EMB_INDEX = 1,     // embedding: token id outside [0, vocab)
  DBG_CE_TARGET = 2,     // cross-entropy: target outside [0, V) and != ignore_index
  DBG_DECODE_POS = 3,    // decode: cache position outside [0, Tmax) or beyond the LDS score buffer
  DBG_ROPE_POS = 4,      // rope: device position negative
};
#ifdef BLLM_KERNEL_DEBUG
#define BLLM_DEBUG_WORD(tu)                                                                        \
  static __device__ unsigned int bllm_dbg_word;                                                     \
  unsigned int debug_take_##tu() {                                                                  \
    unsigned int v = 0, z = 0;                                                                      \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(bllm_dbg_word), sizeof(v)) != hipSuccess) return 0;     \
    if (v) (void)hipMemcpyToSymbol(HIP_SYMBOL(bllm_dbg_word), &z, sizeof(z));                       \
    return v;                                                                                       \
  }
#define BLLM_DASSERT(cond, code)                                   \
  do {                                                             \
    if (!(cond)) atomicCAS(&bllm_dbg_word, 0u, (unsigned)(code));  \
  } while (0)
#else
#define BLLM_DEBUG_WORD(tu) \
  unsigned int debug_take_##tu() { return 0; }
#define BLLM_DASSERT(cond, code) \
  do {                           \
  } while (0)
#endif

}  // namespace bllm

#define BLLM_DISPATCH(dt, T, ...)                                  \
  switch (dt) {                                                    \
    case ::bllm::DType::F32: { typedef float T; __VA_ARGS__; break; }        \
    case ::bllm::DType::BF16: { typedef ::bllm::bf16_t T; __VA_ARGS__; break; } \
    case ::bllm::DType::F16: { typedef ::bllm::f16_t T; __VA_ARGS__; break; }   \
  }
