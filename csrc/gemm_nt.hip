// Forward-layout GEMM on CDNA4 matrix cores: C[M, N] (+)= A[M, K] . B[N, K]^T, both operands
// K-contiguous (a Linear's y = x W^T, and dX = dY W on a transposed weight copy), with optional
// fused epilogues: SwiGLU (Llama gate/up, reference common_components.py:112-124), RoPE (Llama
// QKV, Llama3.py:135-141) and bias + exact GELU (GPT-2 c_fc, GPT2.py:58-62).
//
// One schedule (the losing ones -- one-barrier 8-wave, ping-pong, non-persistent 4-wave, DMA
// cache-policy and barrier-placement variants -- are listed in profiles/r3/kernel_experiments.md
// and profiles/r4/kernel_experiments.md):
//  * tile 256 x 256 x 64 (a K-tile row is one full 128-B line), 4 waves = one per SIMD, each
//    owning 128 x 128 outputs in 64 AGPR accumulators of v_mfma_f32_16x16x32 (operands swapped,
//    so lane l of acc[i][j] holds 4 consecutive columns of one row);
//  * LDS: two buffers of (A image + B image), 32 KiB each, filled by LDS-DMA (buffer_load ...
//    lds, 16 pieces of 1 KiB per wave and K-tile); 16-B chunk c of row r at c ^ ((r >> 1) & 7)
//    (the XOR goes on the per-lane SOURCE offset, the DMA writes lane-linearly): conflict-free
//    ds_read_b128 fragment reads;
//  * per K-tile and wave: 128 MFMAs; the k-step-1 fragments are read over the first 16 MFMAs,
//    the WAR barrier (every wave's reads of the buffer retired) after MFMA 31, the 16 pieces of
//    K-tile t+2 into that buffer one per 5 MFMAs, the RAW barrier (vmcnt: K-tile t+1 landed) at
//    MFMA 112 and the next K-tile's k-step-0 fragments over the last 16; program order pinned
//    with sched_barrier(0) after each MFMA step;
//  * persistent: one workgroup per CU walks output tiles tid, tid + G, ... in an XCD-contiguous,
//    4-deep column-major tile order; the K-tile stream never drains between output tiles (the
//    last two K-tiles of a tile prefetch the next tile's first two) and the epilogue stores
//    straight from the accumulators while the next tile lands in LDS.
#include <stdlib.h>

#include <type_traits>

#include "api.h"
#include "gemm4.h"

namespace bllm {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x8 lds_s16x8;

constexpr int TM = 256, TN = 256, TK = 64;
constexpr int ROWB = TK * 2;             // 128 B per LDS row (one K-tile of one row)
constexpr int IMGB = TM * ROWB;          // 32 KiB per operand image
constexpr int BUFB = 2 * IMGB;           // A + B
constexpr int LDS_BYTES = 2 * BUFB;      // double buffer, 128 KiB
constexpr int GROUP_M = 4;               // tile-group depth (4 measured best of 1-32, profiles/r3)

using g4::EPI_NONE;
using g4::EPI_SWIGLU;
using g4::EPI_ROPE;
using g4::EPI_BIAS_GELU;
using g4::i32x4;
using g4::MfA;
using g4::THREADS4;

// placement of the barriers and DMA pieces in the 128-MFMA K-tile (see the header)
struct Sched4 {
  static constexpr int WAR = 31;                   // barrier after this MFMA
  static constexpr int D0 = WAR + 1, DS = 5;       // first piece, stride
  static constexpr int RAW = 112;                  // before this MFMA (of 128)
  static constexpr int RPM = 1;                    // next-tile fragment reads per MFMA from RAW on
  // piece index issued before/after MFMA m (0..127), -1 if none
  static constexpr int piece(int m) { return m >= D0 && (m - D0) % DS == 0 && (m - D0) / DS < 16 ? (m - D0) / DS : -1; }
};

// EPI_SWIGLU (B = [W_gate; W_up], N = 2F): tile tn covers gate/up column pairs 128tn .. +127;
// the B image interleaves them in 16-row blocks (image rows 128w' + 32b + [0, 16) gate pairs
// 64w' + 16b + [0, 16), the next 16 rows the matching up rows), so a lane's acc[i][2k] and
// acc[i][2k+1] hold 4 gate and the same 4 up columns of one row: the epilogue stores both halves
// of gu and act = silu(g) * u (g, u rounded to T first, as the separate swiglu_fwd kernel).
// EPI_ROPE (the Llama QKV projection, head dim 128 = one wave's 128 columns): columns below nrot
// (the q and k heads) leave rotated, out1 = x1 cos - x2 sin, out2 = x2 cos + x1 sin for the pairs
// (d, d + 64) of the head — acc[i][k] and acc[i][k + 4] of the same lane — at position row % Tq,
// x rounded to T first, exactly as the separate rope_k pass computes it on the stored GEMM output.
// tile -> workgroup maps (experiment knob ``map``, see launch()):
//   0  XCD-contiguous: XCD x walks a contiguous range of the grouped tile order (its own M-band)
//   1  plain: tile order dealt round-robin over the XCDs (what an XCD-unaware launch does)
//   2  XCD-contiguous over the TRANSPOSED grid: each XCD owns an N-band (B private, A shared)
template <typename T, typename OT, bool ACC, int EPI = EPI_NONE>
__global__ __launch_bounds__(THREADS4, 1) void gemm_nt4p_k(const T* __restrict__ A, long lda,
                                                           const T* __restrict__ B, long ldb, OT* __restrict__ C,
                                                           long ldc, int M, int N, int K, OT* __restrict__ act = nullptr,
                                                           int F = 0, const float* __restrict__ cosT = nullptr,
                                                           const float* __restrict__ sinT = nullptr, int Tq = 1,
                                                           int nrot = 0, int group_m = GROUP_M,
                                                           const OT* __restrict__ bias = nullptr, int map = 0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int nbm = M / TM, nbn = N / TN, nblk = nbm * nbn, G = gridDim.x;
  const int q8 = nblk >> 3, r8 = nblk & 7;
  const bool tr = map == 2;
  const int gmaj = tr ? nbn : nbm, gmin = tr ? nbm : nbn, per_group = group_m * gmin;
  auto coords = [&](int tid, long& m0, long& n0) {
    const int xcd = tid & 7;
    const int wid = map == 1 ? tid : (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (tid >> 3);
    const int grp = wid / per_group, first = grp * group_m;
    const int gm = gmaj - first < group_m ? gmaj - first : group_m;
    const int in_g = wid - grp * per_group;
    const int a = first + in_g % gm, b = in_g / gm;
    m0 = (long)(tr ? b : a) * TM;
    n0 = (long)(tr ? a : b) * TN;
  };

  const uint32_t lds0 = lds_u32(smem);
  const uint32_t ldab = (uint32_t)(lda * sizeof(T)), ldbb = (uint32_t)(ldb * sizeof(T));
  uint32_t voA[8], voB[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const uint32_t r = 8u * p + (uint32_t)(lane >> 3), c = 16u * ((lane & 7) ^ ((r >> 1) & 7));
    voA[p] = r * ldab + c;
    if constexpr (EPI == EPI_SWIGLU) {   // image row R -> gate / up row of the tile (see above)
      const uint32_t R = 64u * wave + r, lb = (R & 127) >> 4;
      const uint32_t src = (R >> 7) * 64 + (lb >> 1) * 16 + (R & 15) + ((lb & 1) ? (uint32_t)F : 0u);
      voB[p] = src * ldbb + c;
    } else {
      voB[p] = r * ldbb + c;
    }
  }
  const int nt = K / TK;  // even, >= 2
  constexpr uint32_t TKB = TK * (uint32_t)sizeof(T);
  // B rows a wave stages for the tile at column n0: its 64 contiguous rows, or (SwiGLU) the
  // tile's gate/up pairs n0 / 2 .. (voB carries the row map)
  auto brow = [&](long n0_) -> long { return EPI == EPI_SWIGLU ? n0_ / 2 : n0_ + 64 * wave; };

  int tid = blockIdx.x;
  long m0, n0;
  coords(tid, m0, n0);
  const T* Ac = A + (m0 + 64 * wave) * lda;   // this wave's staged rows of the current tile
  const T* Bc = B + brow(n0) * ldb;
  const T* An = Ac;                           // ... and of the next tile (= current when none)
  const T* Bn = Bc;
  int tid_n = tid + G;
  long m0n = m0, n0n = n0;
  auto set_next = [&]() {
    tid_n = tid + G;
    if (tid_n < nblk) {
      coords(tid_n, m0n, n0n);
      An = A + (m0n + 64 * wave) * lda;
      Bn = B + brow(n0n) * ldb;
    } else {
      An = Ac, Bn = Bc;
    }
  };
  set_next();
  // buffer descriptors of this wave's staged rows: current tile and next tile (uniform, built once
  // per output tile, not per piece)
  i32x4 srAc = g4::make_rsrc(Ac), srBc = g4::make_rsrc(Bc), srAn = g4::make_rsrc(An), srBn = g4::make_rsrc(Bn);
  // descriptors + K offset of the K-tile the pieces of the current step stream (selected once per
  // K-tile by dsel(), placed among the first MFMAs, ahead of the WAR barrier: the pieces behind the
  // barrier then cost one m0 write and the DMA each)
  i32x4 rsA = srAc, rsB = srBc;
  uint32_t soK = 0;
  auto dsel = [&](int t) {   // t: K-tile of the stream (>= nt: the next output tile's t - nt)
    const bool nx = t >= nt;
    const int tt = !nx ? t : (tid_n < nblk ? t - nt : nt - 1);
    const i32x4 a = nx ? srAn : srAc, b = nx ? srBn : srBc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {   // (uniform; pinned to SGPRs for the asm "s" operand)
      rsA[e] = __builtin_amdgcn_readfirstlane(a[e]);
      rsB[e] = __builtin_amdgcn_readfirstlane(b[e]);
    }
    soK = __builtin_amdgcn_readfirstlane((uint32_t)tt * TKB);
  };
  // piece k of the selected K-tile into buffer buf
  auto dmap = [&](int buf, int k) {
    const int p = k & 7;
    const uint32_t d = lds0 + (k >= 8 ? 2 * IMGB : 0) + buf * IMGB + (64 * wave + 8 * p) * ROWB;
    g4::bdma16<1>(k < 8 ? rsA : rsB, k < 8 ? voA[p] : voB[p], soK, d);
  };
  auto dma = [&](int t, int buf, int k) {   // (prologue)
    dsel(t);
    dmap(buf, k);
  };
  const int xo0 = ((0 + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4;
  const int xo1 = ((4 + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4;
  const char* pA0 = smem + (128 * wm + (lane & 15)) * ROWB + xo0;
  const char* pA1 = smem + (128 * wm + (lane & 15)) * ROWB + xo1;
  const char* pB0 = smem + 2 * IMGB + (128 * wn + (lane & 15)) * ROWB + xo0;
  const char* pB1 = smem + 2 * IMGB + (128 * wn + (lane & 15)) * ROWB + xo1;
  auto rdA = [&](int buf, int i, int s) -> s16x8 {
    return *(const lds_s16x8*)((s ? pA1 : pA0) + buf * IMGB + 16 * i * ROWB);
  };
  auto rdB = [&](int buf, int j, int s) -> s16x8 {
    return *(const lds_s16x8*)((s ? pB1 : pB0) + buf * IMGB + 16 * j * ROWB);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{};
  s16x8 a0[8], b0[8], a1[8], b1[8];

#pragma unroll
  for (int k = 0; k < 16; ++k) dma(0, 0, k);
#pragma unroll
  for (int k = 0; k < 16; ++k) dma(1, 1, k);
  wait_vm<16>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = rdA(0, i, 0), b0[i] = rdB(0, i, 0);

  using SC = Sched4;
  // read r (0..15) of a k-step's fragments, in the order the MFMAs consume them
  auto rd16 = [&](s16x8 (&fa)[8], s16x8 (&fb)[8], int buf, int s, int r) {
    if (r == 0) fa[0] = rdA(buf, 0, s);
    else if (r <= 8) fb[r - 1] = rdB(buf, r - 1, s);
    else fa[r - 8] = rdA(buf, r - 8, s);
  };
  auto ktile = [&](int t, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value, nxt = cur ^ 1;
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      const int i = n >> 3, j = n & 7;
      MfA<T>::run(acc[i][j], b0[j], a0[i]);
      if (n < 16) rd16(a1, b1, cur, 1, n);
      if (n == 2) dsel(t + 2);
      if (n == SC::WAR) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      if (SC::piece(n) >= 0) dmap(cur, SC::piece(n));
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      const int i = n >> 3, j = n & 7;
      if (SC::piece(64 + n) >= 0) dmap(cur, SC::piece(64 + n));
      if (64 + n == SC::RAW) {
        wait_vm<16>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      if (64 + n >= SC::RAW && (64 + n - SC::RAW) * SC::RPM < 16) {
#pragma unroll
        for (int q = 0; q < SC::RPM; ++q) rd16(a0, b0, nxt, 0, (64 + n - SC::RAW) * SC::RPM + q);
      }
      MfA<T>::run(acc[i][j], b1[j], a1[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (;;) {
    for (int t = 0; t < nt; t += 2) {
      ktile(t, I0{});
      ktile(t + 1, I1{});
    }
    g4::mfma_drain();
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
    // epilogue straight from the accumulators: acc[i][j] = row 16i + (l & 15), columns
    // 16j + 4(l >> 4) .. +3 of the wave's 128 x 128 block (the accumulate test hoisted out of the
    // element loops: a per-element select makes hipcc branch around every load)
    OT* cw = C + (m0 + 128 * wm + (lane & 15)) * ldc + n0 + 128 * wn + 4 * (lane >> 4);
    auto st4 = [&](OT* o, f32x4 v) {
      if constexpr (sizeof(OT) == 2) {
        typedef OT o4 __attribute__((ext_vector_type(4)));
        *(o4*)o = __builtin_convertvector(v, o4);   // v_cvt_pk_{bf16,f16}_f32 pairs, one 8-B store
      } else {
        *(f32x4*)o = v;
      }
    };
    auto ld4 = [&](const OT* o) -> f32x4 {
      if constexpr (sizeof(OT) == 2) {
        const uint2 u = *(const uint2*)o;
        return f32x4{to_f(__builtin_bit_cast(OT, (short)(u.x & 0xFFFF))), to_f(__builtin_bit_cast(OT, (short)(u.x >> 16))),
                     to_f(__builtin_bit_cast(OT, (short)(u.y & 0xFFFF))), to_f(__builtin_bit_cast(OT, (short)(u.y >> 16)))};
      } else {
        return *(const f32x4*)o;
      }
    };
    // (branch-free: ACC is a template parameter and the host only picks this kernel for rows
    //  aligned to the store width, so hipcc never hoists all 256 accumulator reads above a
    //  branch — which it does otherwise, and spills)
    if constexpr (EPI == EPI_BIAS_GELU) {
      // GPT-2 c_fc: f = acc + bias (rounded to T: the saved pre-activation) and g = GELU(f) with
      // the exact erf form of the separate gelu_fwd kernel (act)
      typedef OT o4 __attribute__((ext_vector_type(4)));
      const long r0 = m0 + 128 * wm + (lane & 15);
      const long cb = n0 + 128 * wn + 4 * (lane >> 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4 bv = __builtin_convertvector(*(const o4*)(bias + cb + 16 * j), f32x4);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const long off = (r0 + 16 * i) * ldc + cb + 16 * j;
          const o4 fb = __builtin_convertvector(acc[i][j] + bv, o4);
          *(o4*)(C + off) = fb;
          o4 gb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = to_f(fb[e]);
            gb[e] = from_f<OT>(gelu_fwd_f<OT>(x));
          }
          *(o4*)(act + off) = gb;
        }
      }
    } else if constexpr (EPI == EPI_ROPE) {
      typedef OT o4 __attribute__((ext_vector_type(4)));
      const long c0 = n0 + 128 * wn;                          // this wave's head
      const bool rot = c0 < nrot;                             // wave-uniform; applied as a select
      const long r0 = m0 + 128 * wm + (lane & 15);
      const int d0 = 4 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const long r = r0 + 16 * i;
        const int pos = (int)(r % Tq);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int d = 16 * k + d0;
          const f32x4 cs = *(const f32x4*)(cosT + (long)pos * 64 + d), sn = *(const f32x4*)(sinT + (long)pos * 64 + d);
          const o4 xa = __builtin_convertvector(acc[i][k], o4), xb = __builtin_convertvector(acc[i][k + 4], o4);
          o4 oa, ob;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x1 = to_f(xa[e]), x2 = to_f(xb[e]);
            const float c = rot ? cs[e] : 1.f, sj = rot ? sn[e] : 0.f;
            oa[e] = from_f<OT>(x1 * c - x2 * sj);
            ob[e] = from_f<OT>(x2 * c + x1 * sj);
          }
          *(o4*)(C + r * ldc + c0 + d) = oa;
          *(o4*)(C + r * ldc + c0 + 64 + d) = ob;
        }
      }
    } else if constexpr (EPI == EPI_SWIGLU) {
      typedef OT o4 __attribute__((ext_vector_type(4)));
      const long g0 = n0 / 2;
      const long r0 = m0 + 128 * wm + (lane & 15);
      const int pc = 64 * wn + 4 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const long r = r0 + 16 * i;
          const long col = g0 + pc + 16 * k;
          const o4 gb = __builtin_convertvector(acc[i][2 * k], o4), ub = __builtin_convertvector(acc[i][2 * k + 1], o4);
          *(o4*)(C + r * ldc + col) = gb;
          *(o4*)(C + r * ldc + F + col) = ub;
          o4 w;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = to_f(gb[e]), b = to_f(ub[e]);
            w[e] = from_f<OT>(a * silu_sig(a) * b);
          }
          *(o4*)(act + r * (long)F + col) = w;
        }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          OT* o = cw + (long)(16 * i) * ldc + 16 * j;
          if constexpr (ACC) st4(o, acc[i][j] + ld4(o));
          else st4(o, acc[i][j]);
        }
    }
    if (tid_n >= nblk) break;
    __builtin_amdgcn_sched_barrier(0);
    {
      // (z through an asm: the zero MFMAs read it as an operand, and a VALU write of an MFMA
      //  operand needs wait states hipcc does not pad for an asm MFMA)
      s16x8 z = s16x8{};
      asm volatile("s_nop 4" : "+v"(z));
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) MfA<T>::zero(acc[i][j], z);
    }
    __builtin_amdgcn_sched_barrier(0);
    // the next tile's first fragments (buffer 0, landed behind the last K-tile's RAW barrier) are
    // read again here so that no fragment register is live across the epilogue
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = rdA(0, i, 0), b0[i] = rdB(0, i, 0);
    tid = tid_n, m0 = m0n, n0 = n0n, Ac = An, Bc = Bn;
    set_next();
    srAc = srAn, srBc = srBn;
    srAn = g4::make_rsrc(An), srBn = g4::make_rsrc(Bn);
  }
  wait_vm0();   // the re-load pieces of the last two stream K-tiles land before the wave ends
}

static int num_cu8() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    ncu = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    ncu = ncu < 8 ? 8 : ncu / 8 * 8;
  }
  return ncu;
}

// persistent grid: one workgroup per CU (a multiple of 8: whole XCDs), or one per tile
inline int grid_of(int M, int N) {
  const int nblk = (M / TM) * (N / TN), ncu = num_cu8();
  return nblk < ncu ? nblk : ncu;
}

template <typename T, typename OT, bool ACC, int EPI>
void set_lds_attr() {
  static const bool at = hipFuncSetAttribute((const void*)gemm_nt4p_k<T, OT, ACC, EPI>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
  (void)at;
}

// tile map (see the kernel) and group depth: the shipped defaults, changed only through
// set_gemm_tile_maps (the round-5 placement A/B, profiles/r5/kernel_experiments.md)
struct NtKnobs {
  int map = 0, gm = GROUP_M;
};
static NtKnobs& knobs() {
  static NtKnobs k;
  return k;
}

template <typename T, typename OT>
void launch(const void* a, long lda, const void* b, long ldb, void* c, long ldc, int M, int N, int K, bool accumulate,
            hipStream_t s) {
  const int grid = grid_of(M, N);
  const NtKnobs& kb = knobs();
  if (accumulate) {
    set_lds_attr<T, OT, true, EPI_NONE>();
    hipLaunchKernelGGL((gemm_nt4p_k<T, OT, true>), dim3(grid), dim3(THREADS4), LDS_BYTES, s, (const T*)a, lda,
                       (const T*)b, ldb, (OT*)c, ldc, M, N, K, nullptr, 0, nullptr, nullptr, 1, 0, kb.gm, nullptr,
                       kb.map);
  } else {
    set_lds_attr<T, OT, false, EPI_NONE>();
    hipLaunchKernelGGL((gemm_nt4p_k<T, OT, false>), dim3(grid), dim3(THREADS4), LDS_BYTES, s, (const T*)a, lda,
                       (const T*)b, ldb, (OT*)c, ldc, M, N, K, nullptr, 0, nullptr, nullptr, 1, 0, kb.gm, nullptr,
                       kb.map);
  }
}

}  // namespace

void set_gemm_nt_tile_map(int map, int group_m) {
  knobs().map = map;
  knobs().gm = group_m > 0 ? group_m : GROUP_M;
}

bool gemm_nt_rope_supported(int M, int N, int K, long lda, long ldb, long ldc, int hd) {
  return hd == 128 && M > 0 && N > 0 && M % TM == 0 && N % TN == 0 && K % (2 * TK) == 0 && ldc % 4 == 0 &&
         (long)TM * lda * 2 < (1L << 31) && (long)TN * ldb * 2 < (1L << 31);
}

void gemm_nt_rope(DType dt, const void* a, long lda, const void* w, long ldw, void* c, long ldc, int M, int N, int K,
                  const float* cosT, const float* sinT, int Tq, int nrot, hipStream_t s) {
  const int grid = grid_of(M, N);
#define BLLM_ROPE4P(TT)                                                                                                \
  do {                                                                                                                 \
    set_lds_attr<TT, TT, false, EPI_ROPE>();                                                                           \
    hipLaunchKernelGGL((gemm_nt4p_k<TT, TT, false, EPI_ROPE>), dim3(grid), dim3(THREADS4), LDS_BYTES, s,               \
                       (const TT*)a, lda, (const TT*)w, ldw, (TT*)c, ldc, M, N, K, (TT*)nullptr, 0, cosT, sinT, Tq,    \
                       nrot);                                                                                          \
  } while (0)
  if (dt == DType::BF16) BLLM_ROPE4P(bf16_t);
  else BLLM_ROPE4P(f16_t);
#undef BLLM_ROPE4P
}

bool gemm_nt_bias_gelu_supported(int M, int N, int K, long lda, long ldb, long ldc) {
  return M > 0 && N > 0 && M % TM == 0 && N % TN == 0 && K % (2 * TK) == 0 && ldc % 4 == 0 &&
         (long)TM * lda * 2 < (1L << 31) && (long)TN * ldb * 2 < (1L << 31);
}

void gemm_nt_bias_gelu(DType dt, const void* a, long lda, const void* w, long ldw, const void* bias, void* f, void* g,
                       long ldc, int M, int N, int K, hipStream_t s) {
  const int grid = grid_of(M, N);
#define BLLM_GELU4P(TT)                                                                                                \
  do {                                                                                                                 \
    set_lds_attr<TT, TT, false, EPI_BIAS_GELU>();                                                                      \
    hipLaunchKernelGGL((gemm_nt4p_k<TT, TT, false, EPI_BIAS_GELU>), dim3(grid), dim3(THREADS4), LDS_BYTES, s,          \
                       (const TT*)a, lda, (const TT*)w, ldw, (TT*)f, ldc, M, N, K, (TT*)g, 0, nullptr, nullptr, 1, 0, \
                       GROUP_M, (const TT*)bias);                                                                            \
  } while (0)
  if (dt == DType::BF16) BLLM_GELU4P(bf16_t);
  else BLLM_GELU4P(f16_t);
#undef BLLM_GELU4P
}

bool gemm_nt2_supported(int M, int N, int K, long lda, long ldb) {
  return M > 0 && N > 0 && K > 0 && M % TM == 0 && N % TN == 0 && K % (2 * TK) == 0 &&
         (long)TM * lda * 2 < (1L << 31) && (long)TN * ldb * 2 < (1L << 31);
}

void gemm_nt2(DType dt, DType odt, const void* a, long lda, const void* b, long ldb, void* c, long ldc, int M, int N,
              int K, bool accumulate, hipStream_t s) {
  BLLM_DISPATCH(odt, OT, {
    if (dt == DType::BF16) launch<bf16_t, OT>(a, lda, b, ldb, c, ldc, M, N, K, accumulate, s);
    else launch<f16_t, OT>(a, lda, b, ldb, c, ldc, M, N, K, accumulate, s);
  });
}

bool gemm_nt_swiglu_supported(int M, int F, int K, long lda, long ldb, long ldgu) {
  return F > 0 && F % 128 == 0 && gemm_nt2_supported(M, 2 * F, K, lda, ldb) && ldgu % 8 == 0;
}

void gemm_nt_swiglu(DType dt, const void* a, long lda, const void* w, long ldw, void* gu, long ldgu, void* act, int M,
                    int F, int K, hipStream_t s) {
  const int grid = grid_of(M, 2 * F);
#define BLLM_SWIGLU4P(TT)                                                                                              \
  do {                                                                                                                 \
    set_lds_attr<TT, TT, false, EPI_SWIGLU>();                                                                         \
    hipLaunchKernelGGL((gemm_nt4p_k<TT, TT, false, EPI_SWIGLU>), dim3(grid), dim3(THREADS4), LDS_BYTES, s,             \
                       (const TT*)a, lda, (const TT*)w, ldw, (TT*)gu, ldgu, M, 2 * F, K, (TT*)act, F);                 \
  } while (0)
  if (dt == DType::BF16) BLLM_SWIGLU4P(bf16_t);
  else BLLM_SWIGLU4P(f16_t);
#undef BLLM_SWIGLU4P
}

}  // namespace bllm
