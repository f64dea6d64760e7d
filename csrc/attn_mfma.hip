// Flash-attention forward on CDNA4 matrix cores (v_mfma_f32_32x32x16_{bf16,f16}).
//
// Replaces the reference's materialised attention (GPT2.py:38-46, Llama3.py:131-155:
// scores [B,H,T,T] -> masked_fill -> softmax -> @V, plus K/V repeat_interleave for GQA).
//
// Formulation ("swapped" operands, so every per-query quantity is lane-local):
//   S^T[key][q] = K · Q^T        A = K tile from LDS (row reads), B = Q fragment in VGPRs
//   O^T[d][q]  += V^T · P^T       A = V^T via ds_read_b64_tr_b16 (hardware transpose),
//                                 B = P taken straight from the S accumulator registers
// With 32x32x16 MFMA the accumulator column is the lane (lane & 31 = query) and its rows
// are keys, so the online-softmax max/sum for a query are a per-lane reduction over its
// 32 registers plus ONE cross-half exchange (lane ^ 32); the rescale of O^T by alpha is
// per lane.  The accumulator registers 8s..8s+7 are reused as the PV B-operand of k-step s
// (element j of lane half h = key 16s + 8(j>>2) + 4h + (j&3)); the V^T operand is read
// with the matching key permutation: two transposed reads of 4 keys each.
//
// Workgroup = 4 waves = 128 queries of one (batch, head); K/V tiles of 64 keys, register
// DMA (global_load_lds) of tile t+1 under the MFMAs of tile t, double-buffered LDS.  GQA reads kv head h / (H/G)
// directly; causal tiles above the diagonal are skipped; q-blocks are launched
// heaviest-first.  LDS images are XOR-swizzled: K in 16-B chunks (conflict-free
// ds_read_b128 row reads), V in 64-B chunks (conflict-free transposed reads).
// Attention-probability dropout (GPT-2) uses the stateless counter hash of common.h.
#include <float.h>
#include "api.h"

namespace bllm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T> struct MF;
template <> struct MF<bf16_t> {
  typedef bf16x8 v8;
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MF<f16_t> {
  typedef f16x8 v8;
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

constexpr float kLog2e = 1.4426950408889634f;
constexpr int FWD_BQ = 128;  // queries per workgroup
constexpr int FWD_BK = 64;   // keys per tile

// ---- swizzled LDS images (byte offsets) -------------------------------------------------
// K: [64 keys][HD] bf16, 16-B chunk c16 of row r stored at chunk c16 ^ swz
template <int HD> __device__ __forceinline__ int k_off(int r, int c16) {
  if constexpr (HD == 128) return r * 256 + ((c16 ^ (r & 15)) << 4);
  else return r * 128 + ((c16 ^ ((r >> 1) & 7)) << 4);
}
// V: [64 keys][HD], 64-B chunk c64 (= 32 columns) of row r stored at c64 ^ swz
template <int HD> __device__ __forceinline__ int v_off(int r, int col) {
  const int c64 = col >> 5, w = (col & 31) << 1;
  if constexpr (HD == 128) return r * 256 + ((c64 ^ (r & 3)) << 6) + w;
  else return r * 128 + ((c64 ^ ((r >> 1) & 1)) << 6) + w;
}

template <typename T> __device__ __forceinline__ uint32_t pack2(float a, float b) {
  T x = from_f<T>(a), y = from_f<T>(b);
  uint16_t ux, uy;
  __builtin_memcpy(&ux, &x, 2);
  __builtin_memcpy(&uy, &y, 2);
  return (uint32_t)ux | ((uint32_t)uy << 16);
}

template <typename T, int HD, bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd_mfma_k(const T* __restrict__ qkv, T* __restrict__ out,
                                                          float* __restrict__ lse, int T_, int H, int G, bool causal,
                                                          uint32_t thr, float inv_keep, uint64_t seed,
                                                          uint64_t doff) {
  typedef typename MF<T>::v8 v8;
  constexpr int KK = HD / 16;               // k-steps of the QK^T product
  constexpr int DT = HD / 32;               // 32-row tiles of O^T
  constexpr int CH = HD / 8;                // 16-B chunks per K/V row
  constexpr int TILE_B = FWD_BK * HD * 2;   // bytes per K (or V) tile
  constexpr int LD = FWD_BK * CH / 256;     // 16-B chunks per thread per tile (K and V each)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nqb = (T_ + FWD_BQ - 1) / FWD_BQ;
  const int qb = nqb - 1 - (int)blockIdx.x;  // heaviest (latest) q-blocks first
  const int h = blockIdx.y, b = blockIdx.z;
  const int g = h / (H / G);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const long rs = (long)(H + 2 * G) * HD;
  const T* qbase = qkv + (long)b * T_ * rs + (long)h * HD;
  const T* kbase = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const T* vbase = qkv + (long)b * T_ * rs + (long)(H + G + g) * HD;
  const int q0 = qb * FWD_BQ;
  const int qi = q0 + w * 32 + l32;  // this lane's query
  const float c = rsqrtf((float)HD) * kLog2e;

  // ---- Q fragments (B operand): Q[qi][16kk + 8hh + 0..7]
  v8 qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    if (qi < T_) qf[kk] = *reinterpret_cast<const v8*>(qbase + (long)qi * rs + kk * 16 + hh * 8);
    else qf[kk] = v8{};
  }

  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x16{};
  float m = -1e30f, l = 0.f;

  const int kend = causal ? min(T_, q0 + FWD_BQ) : T_;
  const int ntiles = (kend + FWD_BK - 1) / FWD_BK;

  // K/V tiles land in LDS by direct DMA (global_load_lds_dwordx4: 1 KiB per wave
  // instruction, lane-linear destination); the XOR swizzle is applied to the per-lane SOURCE
  // address, so the linear DMA image IS the swizzled layout.  No staging VGPRs.
  typedef __attribute__((address_space(3))) void lds_void;
  typedef const __attribute__((address_space(1))) void gbl_void;
  auto issue = [&](int t, int buf) {
    char* kb = smem + buf * 2 * TILE_B;
    char* vb = kb + TILE_B;
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int piece = w * LD + i;             // 1 KiB piece of the 16 KiB tile
      const int P = piece * 64 + lane;          // 16-B chunk position in the image
      const int r = P / CH, pc = P % CH;
      int key = t * FWD_BK + r;
      key = key < T_ ? key : T_ - 1;            // clamp: masked / multiplied by P = 0 later
      int kc16;
      if constexpr (HD == 128) kc16 = pc ^ (r & 15); else kc16 = pc ^ ((r >> 1) & 7);
      const int c64 = (pc >> 2) ^ (HD == 128 ? (r & 3) : ((r >> 1) & 1));
      const int vc16 = c64 * 4 + (pc & 3);
      glds16(kbase + (long)key * rs + kc16 * 8, kb + piece * 1024);
      glds16(vbase + (long)key * rs + vc16 * 8, vb + piece * 1024);
    }
  };

  issue(0, 0);
  wait_vm0();
  __syncthreads();

  const int wq_lo = q0 + w * 32, wq_hi = wq_lo + 31;  // this wave's query range
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) issue(t + 1, buf ^ 1);
    const int k0 = t * FWD_BK;
    const bool active = !causal || k0 <= wq_hi;  // wave-uniform
    if (active) {
      const char* kb = smem + buf * 2 * TILE_B;
      const char* vb = kb + TILE_B;
      // ---- S^T = K Q^T for two 32-key sub-tiles: each sub-tile's K fragments are read
      //      into distinct registers first (one lgkmcnt wait), then the MFMA chain
      f32x16 s[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        v8 ka[KK];
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
          ka[kk] = *reinterpret_cast<const v8*>(kb + k_off<HD>(kt * 32 + l32, kk * 2 + hh));
        __builtin_amdgcn_sched_barrier(0);
        s[kt] = f32x16{};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) s[kt] = MF<T>::mma(ka[kk], qf[kk], s[kt]);
      }
      // ---- scale, mask (selects, no branches), online softmax (lane = query)
      const bool need_mask = (causal && k0 + FWD_BK - 1 > wq_lo) || (k0 + FWD_BK > T_);
      float mx = -INFINITY;
      if (need_mask) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const int kb0 = k0 + kt * 32 + 4 * hh;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kb0 + (r & 3) + 8 * (r >> 2);
            const bool off = (causal & (key > qi)) | (key >= T_);
            const float v = off ? -INFINITY : s[kt][r] * c;
            s[kt][r] = v;
            mx = fmaxf(mx, v);
          }
        }
      } else {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = s[kt][r] * c;
            s[kt][r] = v;
            mx = fmaxf(mx, v);
          }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float alpha = exp2f(m - mn);
      m = mn;
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = exp2f(s[kt][r] - mn);
          ls += p;
          if constexpr (DROP) {
            const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const uint64_t e = (((uint64_t)(b * H + h) * T_ + qi) * T_ + key);
            s[kt][r] = (drop_hash(seed, doff + e) >= thr) ? p * inv_keep : 0.f;
          } else {
            s[kt][r] = p;
          }
        }
      l = l * alpha + ls;
#pragma unroll
      for (int i = 0; i < DT; ++i) o[i] *= alpha;
      // ---- O^T += V^T P^T: P fragments converted just in time from the accumulators,
      //      V^T fragments by hardware-transposed LDS reads
      const int gi = lane & 15, gl = (lane >> 4) & 1;
      const int qrow = gi >> 2, pcol = gi & 3;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          v8 pf;
          {
            uint32_t u[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) u[j] = pack2<T>(s[kt][8 * s2 + 2 * j], s[kt][8 * s2 + 2 * j + 1]);
            __builtin_memcpy(&pf, u, 16);
          }
          const int base = kt * 32 + s2 * 16 + 4 * hh + qrow;
          v8 va[DT];
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const int col = dt * 32 + gl * 16 + pcol * 4;
            const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + v_off<HD>(base, col)));
            const s16x4 r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + v_off<HD>(base + 8, col)));
            short tmp[8] = {r1[0], r1[1], r1[2], r1[3], r2[0], r2[1], r2[2], r2[3]};
            __builtin_memcpy(&va[dt], tmp, 16);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[dt] = MF<T>::mma(va[dt], pf, o[dt]);
        }
    }
    wait_vm0();       // the DMA of tile t+1 has landed (asm-issued, so drained by hand)
    __syncthreads();
  }

  // ---- epilogue: combine the two halves' partial sums, normalise, store O and LSE
  l += __shfl_xor(l, 32, 64);
  if (qi < T_) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    T* orow = out + ((long)b * T_ + qi) * (long)H * HD + (long)h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d0 = dt * 32 + 8 * gq + 4 * hh;
        uint2 v;
        v.x = pack2<T>(o[dt][4 * gq + 0] * inv, o[dt][4 * gq + 1] * inv);
        v.y = pack2<T>(o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d0) = v;
      }
    if (hh == 0) lse[((long)b * H + h) * T_ + qi] = m + log2f(l);
  }
}

bool attn_mfma_head_dim(int hd) { return hd == 64 || hd == 128; }

void attn_fwd_mfma(DType dt, const void* qkv, void* o, float* lse, int B, int T_, int H, int G, int hd, bool causal,
                   float p, uint64_t seed, uint64_t offset, hipStream_t s) {
  const uint32_t thr = drop_threshold(p);
  const float ik = p > 0.f ? 1.f / (1.f - p) : 1.f;
  dim3 grid((T_ + FWD_BQ - 1) / FWD_BQ, H, B), block(256);
#define LAUNCH(TT, HDD)                                                                                       \
  do {                                                                                                        \
    if (p > 0.f)                                                                                              \
      hipLaunchKernelGGL((attn_fwd_mfma_k<TT, HDD, true>), grid, block, 2 * 2 * FWD_BK * HDD * 2, s,          \
                         (const TT*)qkv, (TT*)o, lse, T_, H, G, causal, thr, ik, seed, offset);              \
    else                                                                                                      \
      hipLaunchKernelGGL((attn_fwd_mfma_k<TT, HDD, false>), grid, block, 2 * 2 * FWD_BK * HDD * 2, s,         \
                         (const TT*)qkv, (TT*)o, lse, T_, H, G, causal, thr, ik, seed, offset);              \
  } while (0)
  if (dt == DType::BF16) {
    if (hd == 128) LAUNCH(bf16_t, 128); else LAUNCH(bf16_t, 64);
  } else {
    if (hd == 128) LAUNCH(f16_t, 128); else LAUNCH(f16_t, 64);
  }
#undef LAUNCH
}

}  // namespace bllm
