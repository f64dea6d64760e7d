// Flash attention in fp32 on CDNA4 matrix cores (v_mfma_f32_32x32x2_f32: exact f32 products,
// f32 accumulation, 64 FLOP/clk/SIMD = the f32 vector peak).
//
// The reference's default precision is fp32 and its default model GPT-2 (args.py:77,
// GPT2.py:38-46): scores [B,H,T,T] are materialised, masked, soft-maxed and dropped out.  Here
// the fp32 path is a flash kernel too — O(T) memory at any context length — with the same
// packed-qkv / log2-LSE / counter-hash-dropout contract as the bf16 kernels (attn_mfma.hip), so
// fwd/bwd/recompute share every oracle.
//
// Operand orientation ("swapped", as in the bf16 forward): the query (or, in dK/dV, the key) is
// the accumulator COLUMN = lane & 31, so softmax statistics are lane-local.  A 32x32x2 MFMA
// takes ONE f32 per lane for A and B (lane l: A[l&31][k = l>>5], B[k = l>>5][l&31]); k-step j
// of a head-dim contraction feeds lane half h with dimension h*HD/2 + j, so each lane streams a
// contiguous half-row: Q (or K^T) halves live in VGPRs, K (or Q) rows are read from LDS with
// ds_read_b128 (rows padded by 16 B: the 16 rows of a read group hit 16 distinct bank quads).
// A product that sums over the accumulator's ROW index takes the accumulator register r straight
// as its B operand (lane half h = row (r&3) + 8(r>>2) + 4h), with the A operand read from LDS at
// that row (32 consecutive floats per half: conflict-free ds_read_b32).
//
// Kernels: forward (128 queries / workgroup, 32-key K/V tiles double-buffered through LDS);
// dQ (same tiling, P and dS recomputed from the saved LSE); dK/dV (128 keys / workgroup, loops
// over the query heads of its kv group and 32-query tiles; no atomics, deterministic).
#include <float.h>
#include "api.h"

namespace bllm {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr float kLog2e = 1.4426950408889634f;
constexpr int BQ = 128;  // rows (queries, or keys in dK/dV) per workgroup: 4 waves x 32
constexpr int BT = 32;   // streamed tile (keys, or queries in dK/dV)

__device__ __forceinline__ f32x16 mma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// accumulator register r of lane half h holds row (r&3) + 8(r>>2) + 4h
__device__ __forceinline__ int arow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// [BT rows][HD] fp32 tile: global rows row0.. (clamped to T-1: padded rows are masked by the
// caller), staged in registers and written to a padded LDS image (row stride HD + 4 floats)
template <int HD>
struct TileIO {
  static constexpr int LS = HD + 4;
  static constexpr int CPT = BT * HD / 4 / 256;  // float4 chunks per thread
  f32x4 r[CPT];
  __device__ __forceinline__ void load(const float* base, long rs, int row0, int T_) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = (int)threadIdx.x + i * 256, row = c / (HD / 4), col = (c % (HD / 4)) * 4;
      const int gr = min(row0 + row, T_ - 1);
      r[i] = *reinterpret_cast<const f32x4*>(base + (long)gr * rs + col);
    }
  }
  __device__ __forceinline__ void store(float* lds) const {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = (int)threadIdx.x + i * 256, row = c / (HD / 4), col = (c % (HD / 4)) * 4;
      *reinterpret_cast<f32x4*>(lds + row * LS + col) = r[i];
    }
  }
};

// acc (+)= X[row = lane&31] . Y^T over HD (X rows from padded LDS, Y half-rows in VGPRs)
template <int HD>
__device__ __forceinline__ f32x16 qk(const float* xrow, const float (&y)[HD / 2], f32x16 acc) {
#pragma unroll
  for (int j = 0; j < HD / 2; j += 4) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(xrow + j);
    acc = mma(x[0], y[j], acc);
    acc = mma(x[1], y[j + 1], acc);
    acc = mma(x[2], y[j + 2], acc);
    acc = mma(x[3], y[j + 3], acc);
  }
  return acc;
}

template <int HD>
__device__ __forceinline__ void load_half_row(float (&dst)[HD / 2], const float* row, bool valid) {
#pragma unroll
  for (int j = 0; j < HD / 2; j += 4) {
    const f32x4 v = valid ? *reinterpret_cast<const f32x4*>(row + j) : f32x4{0.f, 0.f, 0.f, 0.f};
    dst[j] = v[0]; dst[j + 1] = v[1]; dst[j + 2] = v[2]; dst[j + 3] = v[3];
  }
}

// ------------------------------------------------------------------------------- forward
template <int HD, bool DROP>
__global__ __launch_bounds__(256) void attn_fwd_f32_k(const float* __restrict__ qkv, float* __restrict__ out,
                                                      float* __restrict__ lse, int T_, int H, int G, int B_,
                                                      bool causal, uint32_t thr, float inv_keep, uint64_t seed,
                                                      uint64_t doff) {
  constexpr int NJ = HD / 2, DT = HD / 32, LS = TileIO<HD>::LS;
  __shared__ __attribute__((aligned(16))) float sK[2][BT * LS];
  __shared__ __attribute__((aligned(16))) float sV[2][BT * LS];
  const int nqb = (T_ + BQ - 1) / BQ, nbh = H * B_, lin = blockIdx.x;
  const int qbi = lin / nbh, bh = lin - qbi * nbh;
  const int qb = causal ? nqb - 1 - qbi : qbi;  // heaviest causal blocks first
  const int h = bh % H, b = bh / H, g = h / (H / G);
  const int lane = threadIdx.x & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const long rs = (long)(H + 2 * G) * HD;
  const float* qbase = qkv + (long)b * T_ * rs + (long)h * HD;
  const float* kbase = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const float* vbase = kbase + (long)G * HD;
  const int q0 = qb * BQ, wq_lo = q0 + w * 32, wq_hi = wq_lo + 31, qi = wq_lo + l32;
  const float c = rsqrtf((float)HD) * kLog2e;
  DropSlab ds;
  uint64_t rowbase = 0;
  if constexpr (DROP) {
    const uint64_t slab = doff + (uint64_t)(b * H + h) * T_ * T_;
    ds.init(seed, slab);
    rowbase = slab + (uint64_t)qi * T_;
  }
  float qf[NJ];
  load_half_row<HD>(qf, qbase + (long)min(qi, T_ - 1) * rs + hh * NJ, qi < T_);
  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x16{};
  float m = -1e30f, l = 0.f;

  const int kend = causal ? min(T_, q0 + BQ) : T_;
  const int ntiles = (kend + BT - 1) / BT;
  const int nact = wq_lo >= T_ ? 0 : (causal ? min(ntiles, wq_hi / BT + 1) : ntiles);
  TileIO<HD> kio, vio;
  kio.load(kbase, rs, 0, T_);
  vio.load(vbase, rs, 0, T_);
  kio.store(sK[0]);
  vio.store(sV[0]);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) {
      kio.load(kbase, rs, (t + 1) * BT, T_);
      vio.load(vbase, rs, (t + 1) * BT, T_);
    }
    if (t < nact) {
      const int k0 = t * BT;
      f32x16 s = qk<HD>(sK[buf] + l32 * LS + hh * NJ, qf, f32x16{});
      if ((causal && k0 + BT - 1 > wq_lo) || k0 + BT > T_ || wq_hi >= T_) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + arow(r, hh);
          if ((causal && key > qi) || key >= T_) s[r] = -INFINITY;
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * c;
      const float mn = fmaxf(m, mx);
      if (__builtin_amdgcn_ballot_w64(mn > m)) {
        const float alpha = exp2f(m - mn);
        l *= alpha;
#pragma unroll
        for (int i = 0; i < DT; ++i) o[i] *= alpha;
        m = mn;
      }
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = exp2f(fmaf(s[r], c, -m));
        ls += p;
        s[r] = p;
      }
      l += ls;
      if constexpr (DROP) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          s[r] = ds.bits16(rowbase + k0 + arow(r, hh)) >= thr ? s[r] * inv_keep : 0.f;
      }
      // O^T += V^T P^T: k-step r pairs keys arow(r, 0) / arow(r, 1) of the two lane halves
      const float* vb = sV[buf] + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float* vr = vb + arow(r, hh) * LS;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] = mma(vr[dt * 32], s[r], o[dt]);
      }
    }
    if (t + 1 < ntiles) {
      kio.store(sK[buf ^ 1]);
      vio.store(sV[buf ^ 1]);
    }
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  if (qi < T_) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    float* orow = out + ((long)b * T_ + qi) * (long)H * HD + (long)h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        *reinterpret_cast<f32x4*>(orow + dt * 32 + 8 * gq + 4 * hh) =
            f32x4{o[dt][4 * gq] * inv, o[dt][4 * gq + 1] * inv, o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv};
    if (hh == 0) lse[((long)b * H + h) * T_ + qi] = m + log2f(l);
  }
}

// ------------------------------------------------------------------------------- dQ
template <int HD, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_dq_f32_k(const float* __restrict__ qkv, const float* __restrict__ lse,
                                                         const float* __restrict__ delta, const float* __restrict__ dout,
                                                         float* __restrict__ dqkv, int T_, int H, int G, int B_,
                                                         bool causal, uint32_t thr, float inv_keep, uint64_t seed,
                                                         uint64_t doff) {
  constexpr int NJ = HD / 2, DT = HD / 32, LS = TileIO<HD>::LS;
  __shared__ __attribute__((aligned(16))) float sK[2][BT * LS];
  __shared__ __attribute__((aligned(16))) float sV[2][BT * LS];
  const int nqb = (T_ + BQ - 1) / BQ, nbh = H * B_, lin = blockIdx.x;
  const int qbi = lin / nbh, bh = lin - qbi * nbh;
  const int qb = causal ? nqb - 1 - qbi : qbi;
  const int h = bh % H, b = bh / H, g = h / (H / G);
  const int lane = threadIdx.x & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const long rs = (long)(H + 2 * G) * HD;
  const float* kbase = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const float* vbase = kbase + (long)G * HD;
  const int q0 = qb * BQ, wq_lo = q0 + w * 32, wq_hi = wq_lo + 31, qi = wq_lo + l32;
  const bool qv = qi < T_;
  const int qc = min(qi, T_ - 1);
  const float scale = rsqrtf((float)HD), c = scale * kLog2e;
  DropSlab ds;
  uint64_t rowbase = 0;
  if constexpr (DROP) {
    const uint64_t slab = doff + (uint64_t)(b * H + h) * T_ * T_;
    ds.init(seed, slab);
    rowbase = slab + (uint64_t)qi * T_;
  }
  float qf[NJ], dof[NJ];
  load_half_row<HD>(qf, qkv + ((long)b * T_ + qc) * rs + (long)h * HD + hh * NJ, qv);
  load_half_row<HD>(dof, dout + ((long)b * T_ + qc) * (long)H * HD + (long)h * HD + hh * NJ, qv);
  const float Lq = qv ? lse[((long)b * H + h) * T_ + qi] : 0.f;
  const float Dq = qv ? delta[((long)b * H + h) * T_ + qi] : 0.f;
  f32x16 dq[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dq[i] = f32x16{};

  const int kend = causal ? min(T_, q0 + BQ) : T_;
  const int ntiles = (kend + BT - 1) / BT;
  const int nact = wq_lo >= T_ ? 0 : (causal ? min(ntiles, wq_hi / BT + 1) : ntiles);
  TileIO<HD> kio, vio;
  kio.load(kbase, rs, 0, T_);
  vio.load(vbase, rs, 0, T_);
  kio.store(sK[0]);
  vio.store(sV[0]);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) {
      kio.load(kbase, rs, (t + 1) * BT, T_);
      vio.load(vbase, rs, (t + 1) * BT, T_);
    }
    if (t < nact) {
      const int k0 = t * BT;
      f32x16 s = qk<HD>(sK[buf] + l32 * LS + hh * NJ, qf, f32x16{});
      f32x16 dp = qk<HD>(sV[buf] + l32 * LS + hh * NJ, dof, f32x16{});
      const bool edge = (causal && k0 + BT - 1 > wq_lo) || k0 + BT > T_ || !qv;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + arow(r, hh);
        float p = exp2f(fmaf(s[r], c, -Lq));
        if (edge && ((causal && key > qi) || key >= T_ || !qv)) p = 0.f;
        float d = dp[r];
        if constexpr (DROP) d = ds.bits16(rowbase + key) >= thr ? d * inv_keep : 0.f;
        s[r] = p * (d - Dq) * scale;  // dS^T
      }
      // dQ^T += K^T dS^T: k-step r, A = K[arow(r, half)][d]
      const float* kb = sK[buf] + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float* kr = kb + arow(r, hh) * LS;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) dq[dt] = mma(kr[dt * 32], s[r], dq[dt]);
      }
    }
    if (t + 1 < ntiles) {
      kio.store(sK[buf ^ 1]);
      vio.store(sV[buf ^ 1]);
    }
    __syncthreads();
  }
  if (qv) {
    float* drow = dqkv + ((long)b * T_ + qi) * rs + (long)h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        *reinterpret_cast<f32x4*>(drow + dt * 32 + 8 * gq + 4 * hh) =
            f32x4{dq[dt][4 * gq], dq[dt][4 * gq + 1], dq[dt][4 * gq + 2], dq[dt][4 * gq + 3]};
  }
}

// ------------------------------------------------------------------------------- dK / dV
template <int HD, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_dkv_f32_k(const float* __restrict__ qkv, const float* __restrict__ lse,
                                                          const float* __restrict__ delta, const float* __restrict__ dout,
                                                          float* __restrict__ dqkv, int T_, int H, int G, int B_,
                                                          bool causal, uint32_t thr, float inv_keep, uint64_t seed,
                                                          uint64_t doff) {
  constexpr int NJ = HD / 2, DT = HD / 32, LS = TileIO<HD>::LS;
  __shared__ __attribute__((aligned(16))) float sQ[2][BT * LS];
  __shared__ __attribute__((aligned(16))) float sO[2][BT * LS];  // dO tile
  __shared__ float sL[2][BT], sD[2][BT];
  const int nbg = G * B_, lin = blockIdx.x;
  const int kbi = lin / nbg, bg = lin - kbi * nbg;  // key block 0 (most causal work) first
  const int g = bg % G, b = bg / G, rep = H / G;
  const int lane = threadIdx.x & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const long rs = (long)(H + 2 * G) * HD, ors = (long)H * HD;
  const int kb0 = kbi * BQ, wk_lo = kb0 + w * 32, kj = wk_lo + l32;
  const bool kv = kj < T_;
  const int kc = min(kj, T_ - 1);
  const float scale = rsqrtf((float)HD), c = scale * kLog2e;
  float kf[NJ], vf[NJ];
  load_half_row<HD>(kf, qkv + ((long)b * T_ + kc) * rs + (long)(H + g) * HD + hh * NJ, kv);
  load_half_row<HD>(vf, qkv + ((long)b * T_ + kc) * rs + (long)(H + G + g) * HD + hh * NJ, kv);
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) { dk[i] = f32x16{}; dv[i] = f32x16{}; }

  const int qstart = causal ? kb0 : 0;
  const int ntq = (T_ - qstart + BT - 1) / BT;
  const int nit = rep * ntq;
  TileIO<HD> qio, oio;
  float lv = 0.f, dv_ = 0.f;
  auto load = [&](int it) {
    const int h = g * rep + it / ntq, qt0 = qstart + (it % ntq) * BT;
    qio.load(qkv + (long)b * T_ * rs + (long)h * HD, rs, qt0, T_);
    oio.load(dout + (long)b * T_ * ors + (long)h * HD, ors, qt0, T_);
    if (threadIdx.x < BT) {
      const int q = qt0 + (int)threadIdx.x;
      // padded query rows: LSE +inf makes P = 0 exactly
      lv = q < T_ ? lse[((long)b * H + h) * T_ + q] : INFINITY;
      dv_ = q < T_ ? delta[((long)b * H + h) * T_ + q] : 0.f;
    }
  };
  auto store = [&](int buf) {
    qio.store(sQ[buf]);
    oio.store(sO[buf]);
    if (threadIdx.x < BT) { sL[buf][threadIdx.x] = lv; sD[buf][threadIdx.x] = dv_; }
  };
  load(0);
  store(0);
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const int buf = it & 1;
    if (it + 1 < nit) load(it + 1);
    const int h = g * rep + it / ntq, qt0 = qstart + (it % ntq) * BT;
    // this wave's keys see queries >= wk_lo only (causal); tiles wholly above are skipped
    if (wk_lo < T_ && (!causal || qt0 + BT - 1 >= wk_lo)) {
      f32x16 s = qk<HD>(sQ[buf] + l32 * LS + hh * NJ, kf, f32x16{});   // S[q][key]
      f32x16 dp = qk<HD>(sO[buf] + l32 * LS + hh * NJ, vf, f32x16{});  // dP[q][key]
      uint64_t slab = 0;
      DropSlab dsl;
      if constexpr (DROP) {
        slab = doff + (uint64_t)(b * H + h) * T_ * T_;
        dsl.init(seed, slab);
      }
      f32x16 pd;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = arow(r, hh), q = qt0 + qr;
        float p = exp2f(fmaf(s[r], c, -sL[buf][qr]));
        if (causal && q < kj) p = 0.f;
        float d = dp[r], pp = p;
        if constexpr (DROP) {
          const bool keep = dsl.bits16(slab + (uint64_t)q * T_ + kj) >= thr;
          pp = keep ? p * inv_keep : 0.f;
          d = keep ? d * inv_keep : 0.f;
        }
        pd[r] = pp;
        s[r] = p * (d - sD[buf][qr]) * scale;  // dS
      }
      const float* qb = sQ[buf] + l32;
      const float* ob = sO[buf] + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = arow(r, hh);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          dv[dt] = mma(ob[qr * LS + dt * 32], pd[r], dv[dt]);  // dV^T += dO^T P
          dk[dt] = mma(qb[qr * LS + dt * 32], s[r], dk[dt]);   // dK^T += Q^T dS
        }
      }
    }
    if (it + 1 < nit) store(buf ^ 1);
    __syncthreads();
  }
  if (kv) {
    float* krow = dqkv + ((long)b * T_ + kj) * rs + (long)(H + g) * HD;
    float* vrow = krow + (long)G * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d = dt * 32 + 8 * gq + 4 * hh;
        *reinterpret_cast<f32x4*>(krow + d) = f32x4{dk[dt][4 * gq], dk[dt][4 * gq + 1], dk[dt][4 * gq + 2], dk[dt][4 * gq + 3]};
        *reinterpret_cast<f32x4*>(vrow + d) = f32x4{dv[dt][4 * gq], dv[dt][4 * gq + 1], dv[dt][4 * gq + 2], dv[dt][4 * gq + 3]};
      }
  }
}

}  // namespace

bool attn_f32_head_dim(int hd) { return hd == 64 || hd == 128; }

#define F32_LAUNCH(KERNEL, GRID)                                                                            \
  do {                                                                                                      \
    if (hd == 128) {                                                                                        \
      if (p > 0.f) hipLaunchKernelGGL((KERNEL<128, true>), GRID, dim3(256), 0, s, ARGS);                    \
      else hipLaunchKernelGGL((KERNEL<128, false>), GRID, dim3(256), 0, s, ARGS);                           \
    } else {                                                                                                \
      if (p > 0.f) hipLaunchKernelGGL((KERNEL<64, true>), GRID, dim3(256), 0, s, ARGS);                     \
      else hipLaunchKernelGGL((KERNEL<64, false>), GRID, dim3(256), 0, s, ARGS);                            \
    }                                                                                                       \
  } while (0)

void attn_fwd_f32(const float* qkv, float* o, float* lse, int B, int T, int H, int G, int hd, bool causal, float p,
                  uint64_t seed, uint64_t offset, hipStream_t s) {
  const uint32_t thr = drop_threshold16(p);
  const float ik = drop_inv_keep(p);
  const dim3 grid(((T + BQ - 1) / BQ) * H * B);
#define ARGS qkv, o, lse, T, H, G, B, causal, thr, ik, seed, offset
  F32_LAUNCH(attn_fwd_f32_k, grid);
#undef ARGS
}

void attn_bwd_f32(const float* qkv, const float* o, const float* lse, const float* dout, float* dqkv, float* delta,
                  int B, int T, int H, int G, int hd, bool causal, float p, uint64_t seed, uint64_t offset,
                  hipStream_t s) {
  const uint32_t thr = drop_threshold16(p);
  const float ik = drop_inv_keep(p);
  attn_delta(DType::F32, o, dout, delta, B, T, H, hd, s);
  const dim3 gq(((T + BQ - 1) / BQ) * H * B), gk(((T + BQ - 1) / BQ) * G * B);
#define ARGS qkv, lse, delta, dout, dqkv, T, H, G, B, causal, thr, ik, seed, offset
  F32_LAUNCH(attn_bwd_dq_f32_k, gq);
  F32_LAUNCH(attn_bwd_dkv_f32_k, gk);
#undef ARGS
}
#undef F32_LAUNCH

}  // namespace bllm
