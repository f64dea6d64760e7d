// Flash-attention backward on CDNA4 matrix cores (v_mfma_f32_32x32x16_{bf16,f16}).
//
// Replaces autograd through the reference's materialised attention (GPT2.py:38-46,
// Llama3.py:131-155) — no [B,H,T,T] tensor, P recomputed from the forward's LSE.
//
// Two atomic-free kernels (dQ is bitwise deterministic):
//  * dK/dV kernel — one workgroup = 4 waves = 128 keys of ONE query head h (kv head
//    g = h / (H/G)).  Key on the MFMA lane: S = Q K^T and dP = dO V^T put the key in the
//    accumulator column, so dV^T += dO^T P and dK^T += Q^T dS take P / dS straight from the
//    accumulator registers as their B operand; dK^T / dV^T for the wave's 32 keys stay in
//    registers for the whole sweep over 32-query steps (one barrier per step).  Per-head
//    partials are plain-stored in fp32 and summed over the H/G heads of each kv group by a
//    tiny reduction (GQA without atomics; MHA writes bf16 directly).
//  * dQ kernel — forward-shaped: one workgroup = 128 queries of one head, the query on the
//    lane (S^T = K Q^T, dP^T = V dO^T), dQ^T += K^T dS^T accumulated in registers over the
//    key tiles, written once.  Costs two extra MFMA products vs. a fused kernel but removes
//    the ~300 MB/layer of fp32 dQ atomics that floored the fused version.
// Softmax constants are lane-local: p = exp2(s*c - lse2), ds = p*(dp - delta)*scale;
// delta = rowsum(dO * O) comes from a pre-pass (attn_naive.hip:attn_delta).  Q/dO (dK/dV
// kernel) and K/V (dQ kernel) tiles arrive by global_load_lds DMA, double-buffered, stored as
// 16-B-chunk XOR images for MFMA row reads and 64-B-chunk XOR images for hardware-transposed
// reads (ds_read_b64_tr_b16).  Causal: only tiles at/below the diagonal; heaviest first.
#include <float.h>
#include "api.h"

namespace bllm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

namespace {
template <typename T> struct MFb;
template <> struct MFb<bf16_t> {
  typedef bf16x8 v8;
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MFb<f16_t> {
  typedef f16x8 v8;
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

// 16-B-chunk XOR image (row reads); rows of HD elements
template <int HD> __device__ __forceinline__ int r_off(int r, int c16) {
  if constexpr (HD == 128) return r * 256 + ((c16 ^ (r & 15)) << 4);
  else return r * 128 + ((c16 ^ ((r >> 1) & 7)) << 4);
}
// 64-B-chunk XOR image (transposed reads); byte offset of element col in row r
template <int HD> __device__ __forceinline__ int t_off(int r, int col) {
  const int c64 = col >> 5, w = (col & 31) << 1;
  if constexpr (HD == 128) return r * 256 + ((c64 ^ (r & 3)) << 6) + w;
  else return r * 128 + ((c64 ^ ((r >> 1) & 1)) << 6) + w;
}
// dS image [32 q][128 keys] bf16: 16-B chunk XOR by q
__device__ __forceinline__ int ds_off(int q, int key) {
  return q * 256 + ((((key >> 3) ^ (q & 15))) << 4) + ((key & 7) << 1);
}

template <typename T> __device__ __forceinline__ uint32_t pk2(float a, float b) {
  T x = from_f<T>(a), y = from_f<T>(b);
  uint16_t ux, uy;
  __builtin_memcpy(&ux, &x, 2);
  __builtin_memcpy(&uy, &y, 2);
  return (uint32_t)ux | ((uint32_t)uy << 16);
}

template <typename v8> __device__ __forceinline__ v8 tr8(const char* base, int off_lo, int off_hi) {
  const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off_lo));
  const s16x4 r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off_hi));
  short tmp[8] = {r1[0], r1[1], r1[2], r1[3], r2[0], r2[1], r2[2], r2[3]};
  v8 a;
  __builtin_memcpy(&a, tmp, 16);
  return a;
}
}  // namespace

constexpr int BWD_BKV = 128;  // keys per workgroup
constexpr int BWD_BQ = 32;    // queries per step
constexpr float kLog2eB = 1.4426950408889634f;

template <typename T, int HD>
__global__ __launch_bounds__(256, (HD == 64 ? 2 : 1)) void attn_bwd_mfma_k(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta, T* __restrict__ dqkv,
                                                          float* __restrict__ dkv_part, int T_, int H, int G,
                                                          bool causal, uint32_t thr, float inv_keep, bool drop,
                                                          uint64_t seed, uint64_t doff) {
  typedef typename MFb<T>::v8 v8;
  constexpr int KK = HD / 16, DT = HD / 32, CH = HD / 8;
  constexpr int IMG = BWD_BQ * HD * 2;          // bytes of one [32][HD] image
  constexpr int PIECES = IMG / 1024;            // 1-KiB DMA pieces per image
  constexpr int BUF = 4 * IMG + 256;            // QR, QT, OR, OT, lse+delta
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* bufs = smem;                            // 2 x BUF

  const int kb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int g = h / (H / G);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const int gi = lane & 15, gl = (lane >> 4) & 1, qrow = gi >> 2, pcol = gi & 3;
  const long rs = (long)(H + 2 * G) * HD;
  const long ors = (long)H * HD;
  const T* qb_ = qkv + (long)b * T_ * rs + (long)h * HD;
  const T* kb_ = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const T* vb_ = qkv + (long)b * T_ * rs + (long)(H + G + g) * HD;
  const T* ob_ = dout + (long)b * T_ * ors + (long)h * HD;
  const float* lse_ = lse + ((long)b * H + h) * T_;
  const float* del_ = delta + ((long)b * H + h) * T_;
  const int k0 = kb * BWD_BKV;
  const int kw0 = k0 + 32 * w;
  const int mykey = kw0 + l32;
  const float scale = rsqrtf((float)HD), c = scale * kLog2eB;

  // ---- K / V fragments of this wave's 32 keys (B operands, key = lane column)
  v8 kf[KK], vf[KK];
  {
    const int kr = mykey < T_ ? mykey : T_ - 1;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      kf[kk] = *reinterpret_cast<const v8*>(kb_ + (long)kr * rs + kk * 16 + hh * 8);
      vf[kk] = *reinterpret_cast<const v8*>(vb_ + (long)kr * rs + kk * 16 + hh * 8);
    }
  }
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) { dk[i] = f32x16{}; dv[i] = f32x16{}; }

  // DMA of one query step (Q and dO, each into a row image and a transposed image) + stats
  auto issue = [&](int q0, int buf) {
    char* base = bufs + buf * BUF;
    for (int pc_ = w; pc_ < 4 * PIECES; pc_ += 4) {
      const int img = pc_ / PIECES, piece = pc_ % PIECES;
      const int P = piece * 64 + lane;
      const int r = P / CH, pc = P % CH;
      int qrow_g = q0 + r;
      qrow_g = qrow_g < T_ ? qrow_g : T_ - 1;
      int c16;
      if ((img & 1) == 0) {  // row image
        if constexpr (HD == 128) c16 = pc ^ (r & 15); else c16 = pc ^ ((r >> 1) & 7);
      } else {               // transposed image
        const int c64 = (pc >> 2) ^ (HD == 128 ? (r & 3) : ((r >> 1) & 1));
        c16 = c64 * 4 + (pc & 3);
      }
      const T* src = (img < 2) ? (qb_ + (long)qrow_g * rs + c16 * 8) : (ob_ + (long)qrow_g * ors + c16 * 8);
      glds16(src, base + img * IMG + piece * 1024);
    }
    if (w == 0) {
      int qq = q0 + (lane & 31);
      qq = qq < T_ ? qq : T_ - 1;
      const float* src = (lane < 32) ? (lse_ + qq) : (del_ + qq);
      glds4(src, base + 4 * IMG);
    }
  };

  const int qstart = causal ? k0 : 0;
  int it = 0;
  if (qstart < T_) issue(qstart, 0);
  wait_vm0();
  __syncthreads();
  for (int q0 = qstart; q0 < T_; q0 += BWD_BQ, ++it) {
    const int buf = it & 1;
    if (q0 + BWD_BQ < T_) issue(q0 + BWD_BQ, buf ^ 1);
    const char* QR = bufs + buf * BUF;
    const char* QT = QR + IMG;
    const char* OR = QR + 2 * IMG;
    const char* OT = QR + 3 * IMG;
    const float* LS = reinterpret_cast<const float*>(QR + 4 * IMG);   // lse[32], delta[32]
    const bool active = (!causal || q0 + BWD_BQ - 1 >= kw0) && kw0 < T_;  // wave-uniform
    if (active) {
      f32x16 sacc = f32x16{}, dpacc = f32x16{};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const v8 aq = *reinterpret_cast<const v8*>(QR + r_off<HD>(l32, kk * 2 + hh));
        sacc = MFb<T>::mma(aq, kf[kk], sacc);
        const v8 ao = *reinterpret_cast<const v8*>(OR + r_off<HD>(l32, kk * 2 + hh));
        dpacc = MFb<T>::mma(ao, vf[kk], dpacc);
      }
      // rows of this lane's accumulator registers: q = q0 + (r&3) + 8(r>>2) + 4hh
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const f32x4 L4 = *reinterpret_cast<const f32x4*>(LS + 8 * gq + 4 * hh);
        const f32x4 D4 = *reinterpret_cast<const f32x4*>(LS + 32 + 8 * gq + 4 * hh);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * gq + j;
          const int q = q0 + 8 * gq + 4 * hh + j;
          float p = exp2f(sacc[r] * c - L4[j]);
          if ((causal && mykey > q) || q >= T_ || mykey >= T_) p = 0.f;
          float dp = dpacc[r], pd = p;
          if (drop) {
            const bool keep = drop_hash(seed, doff + (((uint64_t)(b * H + h) * T_ + q) * T_ + mykey)) >= thr;
            pd = keep ? p * inv_keep : 0.f;
            dp = keep ? dp * inv_keep : 0.f;
          }
          sacc[r] = pd;
          dpacc[r] = p * (dp - D4[j]) * scale;
        }
      }
      // dV^T += dO^T Pd ; dK^T += Q^T dS   (B operands straight from the accumulators)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        v8 pf, df;
        {
          uint32_t u[4], v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            u[j] = pk2<T>(sacc[8 * s2 + 2 * j], sacc[8 * s2 + 2 * j + 1]);
            v[j] = pk2<T>(dpacc[8 * s2 + 2 * j], dpacc[8 * s2 + 2 * j + 1]);
          }
          __builtin_memcpy(&pf, u, 16);
          __builtin_memcpy(&df, v, 16);
        }
        const int base = s2 * 16 + 4 * hh + qrow;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int col = dt * 32 + gl * 16 + pcol * 4;
          const v8 ao = tr8<v8>(OT, t_off<HD>(base, col), t_off<HD>(base + 8, col));
          dv[dt] = MFb<T>::mma(ao, pf, dv[dt]);
          const v8 aq = tr8<v8>(QT, t_off<HD>(base, col), t_off<HD>(base + 8, col));
          dk[dt] = MFb<T>::mma(aq, df, dk[dt]);
        }
      }
    }
    wait_vm0();
    __syncthreads();
  }

  // ---- MHA: write bf16 dK/dV straight into dqkv; GQA: per-head fp32 partials
  if (mykey < T_ && H == G) {
    T* pk = dqkv + ((long)b * T_ + mykey) * rs + (long)(H + g) * HD;
    T* pv = dqkv + ((long)b * T_ + mykey) * rs + (long)(H + G + g) * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d0 = dt * 32 + 8 * gq + 4 * hh;
        uint2 a, bb;
        a.x = pk2<T>(dk[dt][4 * gq], dk[dt][4 * gq + 1]);
        a.y = pk2<T>(dk[dt][4 * gq + 2], dk[dt][4 * gq + 3]);
        bb.x = pk2<T>(dv[dt][4 * gq], dv[dt][4 * gq + 1]);
        bb.y = pk2<T>(dv[dt][4 * gq + 2], dv[dt][4 * gq + 3]);
        *reinterpret_cast<uint2*>(pk + d0) = a;
        *reinterpret_cast<uint2*>(pv + d0) = bb;
      }
  } else if (mykey < T_) {
    const long BT = (long)gridDim.z * T_;
    float* pk = dkv_part + ((long)b * T_ + mykey) * ors + (long)h * HD;
    float* pv = pk + BT * ors;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d0 = dt * 32 + 8 * gq + 4 * hh;
        *reinterpret_cast<f32x4*>(pk + d0) = f32x4{dk[dt][4 * gq], dk[dt][4 * gq + 1], dk[dt][4 * gq + 2], dk[dt][4 * gq + 3]};
        *reinterpret_cast<f32x4*>(pv + d0) = f32x4{dv[dt][4 * gq], dv[dt][4 * gq + 1], dv[dt][4 * gq + 2], dv[dt][4 * gq + 3]};
      }
  }
}

// ---------------------------------------------------------------------------------------
// dQ kernel (forward-shaped): 4 waves x 32 queries of head h; key tiles of 64 by DMA into
// three images per buffer: K rows (S^T = K Q^T), K transposed (dQ^T += K^T dS^T), V rows
// (dP^T = V dO^T).  The query is the lane column, so lse / delta are per-lane scalars.
template <typename T, int HD>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_k(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                        const float* __restrict__ lse,
                                                        const float* __restrict__ delta, T* __restrict__ dqkv,
                                                        int T_, int H, int G, bool causal, uint32_t thr,
                                                        float inv_keep, bool drop, uint64_t seed, uint64_t doff) {
  typedef typename MFb<T>::v8 v8;
  constexpr int BQ = 128, BK = 64;
  constexpr int KK = HD / 16, DT = HD / 32, CH = HD / 8;
  constexpr int IMG = BK * HD * 2;              // bytes of one [64][HD] image
  constexpr int LD = BK * CH / 256;             // 1-KiB pieces per wave per image
  constexpr int BUF = 3 * IMG;                  // K rows, K transposed, V rows
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nqb = (T_ + BQ - 1) / BQ;
  const int qb = nqb - 1 - (int)blockIdx.x;
  const int h = blockIdx.y, b = blockIdx.z;
  const int g = h / (H / G);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const int gi = lane & 15, gl = (lane >> 4) & 1, qrow = gi >> 2, pcol = gi & 3;
  const long rs = (long)(H + 2 * G) * HD;
  const long ors = (long)H * HD;
  const T* kb_ = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const T* vb_ = qkv + (long)b * T_ * rs + (long)(H + G + g) * HD;
  const int q0 = qb * BQ;
  const int qi = q0 + w * 32 + l32;
  const int qc = qi < T_ ? qi : T_ - 1;
  const float scale = rsqrtf((float)HD), c = scale * kLog2eB;

  v8 qf[KK], of[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    qf[kk] = *reinterpret_cast<const v8*>(qkv + ((long)b * T_ + qc) * rs + (long)h * HD + kk * 16 + hh * 8);
    of[kk] = *reinterpret_cast<const v8*>(dout + ((long)b * T_ + qc) * ors + (long)h * HD + kk * 16 + hh * 8);
  }
  const float L = lse[((long)b * H + h) * T_ + qc];
  const float D = delta[((long)b * H + h) * T_ + qc];
  f32x16 dq[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dq[i] = f32x16{};

  auto issue = [&](int t, int buf) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int piece = w * LD + i;
      const int P = piece * 64 + lane;
      const int r = P / CH, pc = P % CH;
      int key = t * BK + r;
      key = key < T_ ? key : T_ - 1;
      int rc16;
      if constexpr (HD == 128) rc16 = pc ^ (r & 15); else rc16 = pc ^ ((r >> 1) & 7);
      const int c64 = (pc >> 2) ^ (HD == 128 ? (r & 3) : ((r >> 1) & 1));
      const int tc16 = c64 * 4 + (pc & 3);
      glds16(kb_ + (long)key * rs + rc16 * 8, base + piece * 1024);
      glds16(kb_ + (long)key * rs + tc16 * 8, base + IMG + piece * 1024);
      glds16(vb_ + (long)key * rs + rc16 * 8, base + 2 * IMG + piece * 1024);
    }
  };

  const int kend = causal ? min(T_, q0 + BQ) : T_;
  const int ntiles = (kend + BK - 1) / BK;
  const int wq_lo = q0 + w * 32, wq_hi = wq_lo + 31;
  issue(0, 0);
  wait_vm0();
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) issue(t + 1, buf ^ 1);
    const int k0 = t * BK;
    if ((!causal || k0 <= wq_hi) && wq_lo < T_) {
      const char* KR = smem + buf * BUF;
      const char* KT = KR + IMG;
      const char* VR = KR + 2 * IMG;
      f32x16 s[2], dp[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x16{};
        dp[kt] = f32x16{};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          const int off = r_off<HD>(kt * 32 + l32, kk * 2 + hh);
          s[kt] = MFb<T>::mma(*reinterpret_cast<const v8*>(KR + off), qf[kk], s[kt]);
          dp[kt] = MFb<T>::mma(*reinterpret_cast<const v8*>(VR + off), of[kk], dp[kt]);
        }
      }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          float p = exp2f(s[kt][r] * c - L);
          if ((causal && key > qi) || key >= T_ || qi >= T_) p = 0.f;
          float d = dp[kt][r];
          if (drop) d = (drop_hash(seed, doff + (((uint64_t)(b * H + h) * T_ + qi) * T_ + key)) >= thr) ? d * inv_keep : 0.f;
          s[kt][r] = p * (d - D) * scale;
        }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          v8 df;
          {
            uint32_t u[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) u[j] = pk2<T>(s[kt][8 * s2 + 2 * j], s[kt][8 * s2 + 2 * j + 1]);
            __builtin_memcpy(&df, u, 16);
          }
          const int base = kt * 32 + s2 * 16 + 4 * hh + qrow;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const int col = dt * 32 + gl * 16 + pcol * 4;
            const v8 a = tr8<v8>(KT, t_off<HD>(base, col), t_off<HD>(base + 8, col));
            dq[dt] = MFb<T>::mma(a, df, dq[dt]);
          }
        }
    }
    wait_vm0();
    __syncthreads();
  }
  if (qi < T_) {
    T* row = dqkv + ((long)b * T_ + qi) * rs + (long)h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d0 = dt * 32 + 8 * gq + 4 * hh;
        uint2 v;
        v.x = pk2<T>(dq[dt][4 * gq], dq[dt][4 * gq + 1]);
        v.y = pk2<T>(dq[dt][4 * gq + 2], dq[dt][4 * gq + 3]);
        *reinterpret_cast<uint2*>(row + d0) = v;
      }
  }
}

// GQA: dqkv[:, k/v part] = bf16(sum over the H/G query heads of each kv group)
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_kv_reduce_k(const float* __restrict__ dkv_part, T* __restrict__ dqkv,
                                                            long BT, int H, int G, int HD) {
  const int rep = H / G;
  const long rs = (long)(H + 2 * G) * HD;
  const long per_row = 2L * G * HD / 4;
  const long total = BT * per_row;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long row = i / per_row;
    const int kvcol = (int)(i - row * per_row) * 4;  // in [0, 2*G*HD)
    const int which = kvcol / (G * HD);
    const int gg = (kvcol % (G * HD)) / HD, d = kvcol % HD;
    const float* src = dkv_part + (long)which * BT * H * HD + row * H * HD;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < rep; ++r) {
      const float4 x = *reinterpret_cast<const float4*>(src + (long)(gg * rep + r) * HD + d);
      v[0] += x.x; v[1] += x.y; v[2] += x.z; v[3] += x.w;
    }
    T* dst = dqkv + row * rs + (long)H * HD + kvcol;
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = from_f<T>(v[j]);
  }
}

void attn_bwd_mfma(DType dt, const void* qkv, const void* o, const float* lse, const void* dout, void* dqkv,
                   float* delta, float* dq_acc, float* dkv_part, int B, int T_, int H, int G, int hd, bool causal,
                   float p, uint64_t seed, uint64_t offset, hipStream_t s) {
  (void)dq_acc;
  const uint32_t thr = drop_threshold(p);
  const float ik = p > 0.f ? 1.f / (1.f - p) : 1.f;
  attn_delta(dt, o, dout, delta, B, T_, H, hd, s);
  dim3 grid_kv((T_ + BWD_BKV - 1) / BWD_BKV, H, B), grid_q((T_ + 127) / 128, H, B), block(256);
  auto lds_kv = [](int HD) { return 2 * (4 * BWD_BQ * HD * 2 + 256); };
  auto lds_q = [](int HD) { return 2 * 3 * 64 * HD * 2; };
#define LAUNCH(TT, HDD)                                                                                         \
  do {                                                                                                          \
    hipLaunchKernelGGL((attn_bwd_mfma_k<TT, HDD>), grid_kv, block, lds_kv(HDD), s, (const TT*)qkv,            \
                       (const TT*)dout, lse, delta, (TT*)dqkv, dkv_part, T_, H, G, causal, thr, ik, p > 0.f,    \
                       seed, offset);                                                                           \
    hipLaunchKernelGGL((attn_bwd_dq_k<TT, HDD>), grid_q, block, lds_q(HDD), s, (const TT*)qkv,                 \
                       (const TT*)dout, lse, delta, (TT*)dqkv, T_, H, G, causal, thr, ik, p > 0.f, seed,       \
                       offset);                                                                                 \
  } while (0)
  if (dt == DType::BF16) {
    if (hd == 128) LAUNCH(bf16_t, 128); else LAUNCH(bf16_t, 64);
  } else {
    if (hd == 128) LAUNCH(f16_t, 128); else LAUNCH(f16_t, 64);
  }
#undef LAUNCH
  if (H != G) {
    const long BT = (long)B * T_;
    const long groups = BT * 2L * G * hd / 4;
    const int fg = (int)((groups + 255) / 256 < 4096 ? (groups + 255) / 256 : 4096);
    BLLM_DISPATCH(dt, TT, {
      hipLaunchKernelGGL(attn_bwd_kv_reduce_k<TT>, dim3(fg), dim3(256), 0, s, dkv_part, (TT*)dqkv, BT, H, G, hd);
    });
  }
}

}  // namespace bllm
