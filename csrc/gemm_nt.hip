// Forward-layout GEMM on CDNA4 matrix cores: C[M, N] (+)= A[M, K] . B[N, K]^T, both operands
// K-contiguous (a Linear's y = x W^T, and dX = dY W on a transposed weight copy).
//
// Why a second kernel next to csrc/gemm_wgrad.hip: that kernel stages 32-deep k-slots, which
// for K-contiguous operands means 64-B row segments per slot (half a 128-B line per request),
// and runs this layout at 1.19-1.28 PF against hipBLASLt's 1.46-1.60 PF
// (profiles/r2_gemm_nt_vs_hipblaslt.jsonl).  Here every K-tile is 64 deep, so each staged row
// is one full 128-B line:
//
//  * tile 256 x 256 x 64, 8 waves = 2 (M) x 4 (N), 128 x 64 outputs per wave in four
//    quadrants of 64 x 32 (acc[8][4] of v_mfma_f32_16x16x32 results);
//  * LDS: two buffers of (A image + B image), 32 KiB each, 128 KiB total, filled by LDS-DMA
//    (global_load_lds_dwordx4, 8 per lane per K-tile, 1 KiB = 8 rows per wave instruction);
//    16-B chunk c of row r stored at c ^ ((r >> 1) & 7) (the XOR goes on the per-lane global
//    SOURCE address; the DMA writes LDS lane-linearly) -- conflict-free ds_read_b128 fragment
//    reads for all four 16-lane groups of the instruction;
//  * schedule per K-tile t (one barrier):  P0: read A(qm1), B(qn1) of t; MFMA (qm0, qn0)
//    P1: MFMA (qm0, qn1) | wait own DMA of t+1 + own LDS reads, s_barrier, DMA t+2 into the
//    buffer of t | P2: read A(qm0) of t+1; MFMA (qm1, qn1) | P3: read B(qn0) of t+1; MFMA
//    (qm1, qn0).  The DMA of a K-tile is issued a full K-tile (64 MFMAs per wave) before its
//    first read; fragments are read one phase before their MFMAs; B register sets swap roles
//    every tile (loop unrolled by two);
//  * blockIdx -> tile: XCD-contiguous ranges (bijective), GROUP_M-deep column-major groups;
//  * epilogue through LDS in two 128-row passes, 16-B row-contiguous stores (+ the old C when
//    accumulating).
#include <stdlib.h>

#include <type_traits>

#include "api.h"
#include "gemm4.h"

namespace bllm {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x8 lds_s16x8;

template <typename T> struct Mf;
template <> struct Mf<bf16_t> {
  static __device__ __forceinline__ f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
};
template <> struct Mf<f16_t> {
  static __device__ __forceinline__ f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
  }
};

constexpr int TM = 256, TN = 256, TK = 64;
constexpr int ROWB = TK * 2;             // 128 B per LDS row (one K-tile of one row)
constexpr int IMGB = TM * ROWB;          // 32 KiB per operand image
constexpr int BUFB = 2 * IMGB;           // A + B
constexpr int LDS_BYTES = 2 * BUFB;      // double buffer, 128 KiB
constexpr int THREADS = 512;
constexpr int GROUP_M = 8;

// one quadrant's fragments: A 4 m-frags x 2 k-steps, B 2 n-frags x 2 k-steps
struct FA { s16x8 f[4][2]; };
struct FB { s16x8 f[2][2]; };

// EPI_SWIGLU: B = [W_gate; W_up] ([2F, K]); tile tn takes gate rows 128tn.. and up rows F + 128tn..
// (image rows 0-127 / 128-255), the epilogue stores gu (both halves, as the plain GEMM would) and
// act = silu(g) * u for its 128 columns, rounded exactly like the separate SwiGLU kernel
// (elementwise.hip: g, u rounded to T first, then a / (1 + exp(-a)) * u in fp32).
using g4::EPI_NONE;
using g4::EPI_SWIGLU;
using g4::EPI_ROPE;
using g4::EPI_BIAS_GELU;
using g4::i32x4;
using g4::MfA;
using g4::THREADS4;

// ---- epilogue: lane holds C[16I + 4(l>>4) + e][16J + (l&15)] of its wave's 128 x 64 block
template <typename T, typename OT, int EPI>
__device__ __forceinline__ void epilogue(f32x4 (&acc)[8][4], char* smem, int wm, int wn, int lane, OT* C, long ldc,
                                         long m0, long n0, long g0, long u0, int accumulate, int wide, OT* act,
                                         int F) {
  OT* cbase = C + m0 * ldc + n0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (wide) {
    constexpr int RB = TN * 4;                // fp32 row of the tile in LDS
    constexpr int EPT = 16 / (int)sizeof(OT);
    constexpr int NCH = EPT / 4;
    constexpr int IPR = TN / EPT;
    constexpr int TRIPS = 128 * IPR / THREADS;
    struct alignas(16) V16 { OT e[EPT]; };
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (wm == pass) {
#pragma unroll
        for (int I = 0; I < 8; ++I)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int J = 0; J < 4; ++J) {
              const int lr = 16 * I + 4 * (lane >> 4) + e, col = wn * 64 + 16 * J + (lane & 15);
              *(float*)(smem + lr * RB + ((((col >> 2) ^ (lr & 7)) << 4) | ((col & 3) << 2))) = acc[I][J][e];
            }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int tr = 0; tr < TRIPS; ++tr) {
        const int q = (int)threadIdx.x + tr * THREADS;
        const int lr = q / IPR, it = q % IPR;
        float v[EPT];
#pragma unroll
        for (int h = 0; h < NCH; ++h) {
          const f32x4 x = *(const f32x4*)(smem + lr * RB + (((it * NCH + h) ^ (lr & 7)) << 4));
#pragma unroll
          for (int k = 0; k < 4; ++k) v[4 * h + k] = x[k];
        }
        long col = it * EPT;
        if constexpr (EPI == EPI_SWIGLU) col = col < 128 ? g0 + col - n0 : u0 + (col - 128) - n0;
        V16* o = (V16*)(cbase + (long)(pass * 128 + lr) * ldc + col);
        if (accumulate) {
          const V16 old = *o;
#pragma unroll
          for (int k = 0; k < EPT; ++k) v[k] += to_f(old.e[k]);
        }
        V16 w;
#pragma unroll
        for (int k = 0; k < EPT; ++k) w.e[k] = from_f<OT>(v[k]);
        *o = w;
      }
      if constexpr (EPI == EPI_SWIGLU) {
        // act[row][g0 + c] = silu(g) * u for the tile's 128 gate / up column pairs
        constexpr int AIPR = 128 / EPT;
        constexpr int ATRIPS = 128 * AIPR / THREADS;
#pragma unroll
        for (int tr = 0; tr < ATRIPS; ++tr) {
          const int q = (int)threadIdx.x + tr * THREADS;
          const int lr = q / AIPR, it = q % AIPR;
          float g[EPT], u[EPT];
#pragma unroll
          for (int h = 0; h < NCH; ++h) {
            const f32x4 xg = *(const f32x4*)(smem + lr * RB + (((it * NCH + h) ^ (lr & 7)) << 4));
            const f32x4 xu = *(const f32x4*)(smem + lr * RB + (((32 + it * NCH + h) ^ (lr & 7)) << 4));
#pragma unroll
            for (int k = 0; k < 4; ++k) g[4 * h + k] = xg[k], u[4 * h + k] = xu[k];
          }
          V16 w;
#pragma unroll
          for (int k = 0; k < EPT; ++k) {
            const float a = to_f(from_f<OT>(g[k])), b = to_f(from_f<OT>(u[k]));
            w.e[k] = from_f<OT>(a / (1.f + __expf(-a)) * b);
          }
          *(V16*)(act + (m0 + pass * 128 + lr) * (long)F + g0 + it * EPT) = w;
        }
      }
      if (pass == 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    }
    return;
  }
  OT* c = cbase + (128 * wm + 4 * (lane >> 4)) * ldc + 64 * wn + (lane & 15);
  if (accumulate) {
#pragma unroll
    for (int I = 0; I < 8; ++I)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int J = 0; J < 4; ++J) {
          OT* o = c + (long)(16 * I + e) * ldc + 16 * J;
          *o = from_f<OT>(to_f(*o) + acc[I][J][e]);
        }
  } else {
#pragma unroll
    for (int I = 0; I < 8; ++I)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int J = 0; J < 4; ++J) c[(long)(16 * I + e) * ldc + 16 * J] = from_f<OT>(acc[I][J][e]);
  }
}

template <typename T, typename OT, int EPI>
__global__ __launch_bounds__(THREADS) void gemm_nt_k(const T* __restrict__ A, long lda, const T* __restrict__ B,
                                                     long ldb, OT* __restrict__ C, long ldc, int M, int N, int K,
                                                     int accumulate, int wide, OT* __restrict__ act, int F) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 2, wn = wave & 3;

  // ---- tile id: XCD-contiguous (bijective), then GROUP_M-deep column-major groups
  const int nbm = M / TM, nbn = N / TN, nblk = nbm * nbn;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int per_group = GROUP_M * nbn;
  const int grp = wid / per_group;
  const int first_m = grp * GROUP_M;
  const int gm = nbm - first_m < GROUP_M ? nbm - first_m : GROUP_M;
  const int in_g = wid - grp * per_group;
  const int tm = first_m + in_g % gm, tn = in_g / gm;
  const long m0 = (long)tm * TM, n0 = (long)tn * TN;

  // ---- staging: wave w moves rows 32w .. 32w+31 of both images (4 x 1 KiB pieces each);
  //      lane -> row 8i + l/8 of the piece, physical chunk l%8, logical chunk p ^ ((row>>1)&7)
  // (offsets recomputed per issue from an opaque copy of the lane id: a few full-rate VALU
  //  instead of 8 VGPRs held across the loop, which the accumulators need)
  const uint32_t lds0 = lds_u32(smem);
  // this wave's 32 rows of each image (image rows 32w .. 32w + 31)
  const long g0 = (long)tn * 128, u0 = (long)F + (long)tn * 128;  // EPI_SWIGLU column bases
  const long brow0 = EPI == EPI_SWIGLU ? (wave < 4 ? g0 + 32 * wave : u0 + 32 * (wave - 4)) : n0 + 32 * wave;
  const T* Abase = A + (m0 + 32 * wave) * lda;
  const T* Bbase = B + brow0 * ldb;
  const uint32_t ldab = (uint32_t)(lda * sizeof(T)), ldbb = (uint32_t)(ldb * sizeof(T));
  auto stage = [&](int t, int buf) {
    const void* a = sgpr_ptr(Abase + (long)t * TK);
    const void* b = sgpr_ptr(Bbase + (long)t * TK);
    const uint32_t d = lds0 + buf * BUFB + wave * 4 * 1024;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // local row r (image row 32w + r: same XOR, 32w is a multiple of 16)
      const uint32_t r = 8 * i + (ln >> 3), c = (ln & 7) ^ ((r >> 1) & 7);
      glds16s(a, r * ldab + 16 * c, d + i * 1024);
      glds16s(b, r * ldbb + 16 * c, d + IMGB + i * 1024);
    }
  };

  // ---- fragment read offsets: lane reads row (.. + (l & 15)), logical chunk 4s + (l >> 4)
  const int xo0 = ((0 + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4;
  const int xo1 = ((4 + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4;
  const int arow = (128 * wm + (lane & 15)) * ROWB;
  const int brow = IMGB + (64 * wn + (lane & 15)) * ROWB;
  auto rdA = [&](FA& F, int buf, int qm) {
    const char* base = smem + buf * BUFB + arow + (64 * qm) * ROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      F.f[i][0] = *(const lds_s16x8*)(base + 16 * i * ROWB + xo0);
      F.f[i][1] = *(const lds_s16x8*)(base + 16 * i * ROWB + xo1);
    }
  };
  auto rdB = [&](FB& F, int buf, int qn) {
    const char* base = smem + buf * BUFB + brow + (32 * qn) * ROWB;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      F.f[j][0] = *(const lds_s16x8*)(base + 16 * j * ROWB + xo0);
      F.f[j][1] = *(const lds_s16x8*)(base + 16 * j * ROWB + xo1);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};
  auto mma = [&](const FA& a, const FB& b, int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * qm + i][2 * qn + j] = Mf<T>::run(a.f[i][s], b.f[j][s], acc[4 * qm + i][2 * qn + j]);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nt = K / TK;  // even (host: K % 128 == 0)
  stage(0, 0);
  if (nt > 1) stage(1, 1);
  if (nt > 1) wait_vm<8>(); else wait_vm0();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  FA A0, A1;
  FB Bp, Bq;
  rdA(A0, 0, 0);
  rdB(Bp, 0, 0);

  // one K-tile; X = the B set holding qn0 of tile t on entry (the other receives qn1, then
  // qn0 of tile t+1)
  auto tile = [&](int t, FB& X, FB& Y) {
    const int cur = t & 1, nxt = cur ^ 1;
    const bool more = t + 1 < nt;
    // P0: fragments of (qm1, qn1) for P1-P3; MFMA (qm0, qn0)
    rdB(Y, cur, 1);
    rdA(A1, cur, 1);
    mma(A0, X, 0, 0);
    // P1: MFMA (qm0, qn1)
    mma(A0, Y, 0, 1);
    // sync: own reads of buffer cur retired, own DMA of tile t+1 landed; after the barrier every
    // wave is past both, so tile t+1 is readable and buffer cur can take tile t+2
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_vm0();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < nt) stage(t + 2, cur);
    // P2: A(qm0) of t+1; MFMA (qm1, qn1)
    if (more) rdA(A0, nxt, 0);
    mma(A1, Y, 1, 1);
    // P3: B(qn0) of t+1 into Y; MFMA (qm1, qn0)
    mma(A1, X, 1, 0);
    if (more) rdB(Y, nxt, 0);
  };
  for (int t = 0; t < nt; t += 2) {
    tile(t, Bp, Bq);
    tile(t + 1, Bq, Bp);
  }

  epilogue<T, OT, EPI>(acc, smem, wm, wn, lane, C, ldc, m0, n0, g0, u0, accumulate, wide, act, F);
}

// ---- ping-pong schedule (BLLM_GEMM_NT_SCHED=1): same tile, waves, LDS images and epilogue;
// the two wave rows (wm = 0: waves 0-3, wm = 1: waves 4-7, one of each per SIMD) run one
// barrier apart, so on every SIMD one wave is in its 16-MFMA block while the other issues its
// fragment reads and LDS-DMA and waits.  Per K-tile, four phases, one C quadrant each:
//   phase 1 (qm0, qn0): read A(qm0) + B(qn0)   phase 2 (qm0, qn1): read B(qn1)
//   phase 3 (qm1, qn1): read A(qm1)            phase 4 (qm1, qn0): no reads (B(qn0) kept)
// and each phase = [reads] [2 LDS-DMA of one staged quarter] vmcnt(8) barrier lgkmcnt(0)
// [16 MFMA] barrier.  Staging is by quarter (16 KiB: the A rows of one qm, or the B rows of one
// qn, over the whole tile), in the order the phases consume them, each into the buffer of its
// K-tile's parity: quarter sequence 4t + {0: A qm0, 1: B qn0, 2: B qn1, 3: A qm1}; quarter s is
// issued in the phase 4 phases before the one whose reads retire it, i.e. with 4 quarters
// (8 DMA per wave) in flight behind it: every phase waits vmcnt(8) (fewer in the tail).
// RAW: a quarter is read only in a phase after the barrier that follows every wave's wait for
// it (the stagger moves the other row's wait one barrier EARLIER, never later).  WAR: a slot is
// refilled >= 2 phases after its last read, whose lgkmcnt(0) precedes an intervening barrier.
template <typename T, typename OT, int EPI>
__global__ __launch_bounds__(THREADS) void gemm_nt_pp_k(const T* __restrict__ A, long lda, const T* __restrict__ B,
                                                        long ldb, OT* __restrict__ C, long ldc, int M, int N, int K,
                                                        int accumulate, int wide, OT* __restrict__ act, int F) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 2, wn = wave & 3;

  const int nbm = M / TM, nbn = N / TN, nblk = nbm * nbn;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int per_group = GROUP_M * nbn;
  const int grp = wid / per_group;
  const int first_m = grp * GROUP_M;
  const int gm = nbm - first_m < GROUP_M ? nbm - first_m : GROUP_M;
  const int in_g = wid - grp * per_group;
  const int tm = first_m + in_g % gm, tn = in_g / gm;
  const long m0 = (long)tm * TM, n0 = (long)tn * TN;
  const long g0 = (long)tn * 128, u0 = (long)F + (long)tn * 128;

  const uint32_t lds0 = lds_u32(smem);
  const uint32_t ldab = (uint32_t)(lda * sizeof(T)), ldbb = (uint32_t)(ldb * sizeof(T));
  const int nt = K / TK;
  // quarter k of K-tile t: this wave moves 8-row groups 2w, 2w+1 of the quarter's 128 rows
  auto stageq = [&](int t, int k) {
    const int buf = t & 1;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int g = 2 * wave + j;
      const void* src;
      uint32_t ld, dst;
      int r0;
      if (k == 0 || k == 3) {  // A rows 128 (g>>3) + 64 qm + 8 (g&7) ..
        r0 = 128 * (g >> 3) + 64 * (k == 3) + 8 * (g & 7);
        src = sgpr_ptr(A + (m0 + r0) * lda + (long)t * TK);
        ld = ldab;
        dst = lds0 + buf * BUFB + r0 * ROWB;
      } else {                 // B rows 64 (g>>2) + 32 qn + 8 (g&3) ..
        r0 = 64 * (g >> 2) + 32 * (k == 2) + 8 * (g & 3);
        const long br = EPI == EPI_SWIGLU ? (r0 < 128 ? g0 + r0 : u0 + (r0 - 128)) : n0 + r0;
        src = sgpr_ptr(B + br * ldb + (long)t * TK);
        ld = ldbb;
        dst = lds0 + buf * BUFB + IMGB + r0 * ROWB;
      }
      // image row r0 + l/8, physical chunk l%8 holds logical chunk p ^ ((row >> 1) & 7)
      const uint32_t r = (uint32_t)(ln >> 3), c = (ln & 7) ^ (((r0 + r) >> 1) & 7);
      glds16s(src, r * ld + 16 * c, dst);
    }
  };

  const int xo0 = ((0 + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4;
  const int xo1 = ((4 + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4;
  const int arow = (128 * wm + (lane & 15)) * ROWB;
  const int brow = IMGB + (64 * wn + (lane & 15)) * ROWB;
  auto rdA = [&](FA& Fr, int buf, int qm) {
    const char* base = smem + buf * BUFB + arow + (64 * qm) * ROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      Fr.f[i][0] = *(const lds_s16x8*)(base + 16 * i * ROWB + xo0);
      Fr.f[i][1] = *(const lds_s16x8*)(base + 16 * i * ROWB + xo1);
    }
  };
  auto rdB = [&](FB& Fr, int buf, int qn) {
    const char* base = smem + buf * BUFB + brow + (32 * qn) * ROWB;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      Fr.f[j][0] = *(const lds_s16x8*)(base + 16 * j * ROWB + xo0);
      Fr.f[j][1] = *(const lds_s16x8*)(base + 16 * j * ROWB + xo1);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  // the quarter with sequence s (4t + k) is issued iff t < nt; when phase p of tile t waits, the
  // newest issued quarter is min(iss, 4 nt - 1) and the one it must retire is req
  auto wait_for = [&](int iss, int req) {
    const int last = 4 * nt - 1;
    const int n = 2 * ((iss < last ? iss : last) - req);
    if (n >= 8) wait_vm<8>();
    else if (n == 6) wait_vm<6>();
    else if (n == 4) wait_vm<4>();
    else if (n == 2) wait_vm<2>();
    else wait_vm0();
  };
  auto sync_mma = [&](const FA& a, const FB& b, int qm, int qn) {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * qm + i][2 * qn + j] = Mf<T>::run(a.f[i][s], b.f[j][s], acc[4 * qm + i][2 * qn + j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // prologue: quarters 0..5 (tile 0 and A qm0 / B qn0 of tile 1), retire quarters 0, 1
  stageq(0, 0);
  stageq(0, 1);
  stageq(0, 2);
  stageq(0, 3);
  if (nt > 1) {
    stageq(1, 0);
    stageq(1, 1);
  }
  wait_for(5, 1);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (wm == 1) {  // the stagger: row 1 runs one barrier behind row 0
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  FA a;
  FB b0, b1;
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    // phase 1: (qm0, qn0); stage B qn1 of t+1; retire B qn1 of t (read in phase 2)
    rdA(a, cur, 0);
    rdB(b0, cur, 0);
    if (t + 1 < nt) stageq(t + 1, 2);
    wait_for(4 * (t + 1) + 2, 4 * t + 2);
    sync_mma(a, b0, 0, 0);
    // phase 2: (qm0, qn1); stage A qm1 of t+1
    rdB(b1, cur, 1);
    if (t + 1 < nt) stageq(t + 1, 3);
    wait_for(4 * (t + 1) + 3, 4 * t + 3);
    sync_mma(a, b1, 0, 1);
    // phase 3: (qm1, qn1); stage A qm0 of t+2
    rdA(a, cur, 1);
    if (t + 2 < nt) stageq(t + 2, 0);
    wait_for(4 * (t + 2), 4 * (t + 1));
    sync_mma(a, b1, 1, 1);
    // phase 4: (qm1, qn0), no reads; stage B qn0 of t+2
    if (t + 2 < nt) stageq(t + 2, 1);
    wait_for(4 * (t + 2) + 1, 4 * (t + 1) + 1);
    sync_mma(a, b0, 1, 0);
  }
  if (wm == 0) {  // balance the stagger
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  epilogue<T, OT, EPI>(acc, smem, wm, wn, lane, C, ldc, m0, n0, g0, u0, accumulate, wide, act, F);
}

// ---- 4-wave schedule (BLLM_GEMM_NT_SCHED=2): the same 256 x 256 x 64 tile, LDS images and
// swizzle on 4 waves (one per SIMD) of 128 x 128 outputs each (acc[8][8]: 256 accumulator
// registers, which the compiler places in AGPRs), the layout gfx950's hipBLASLt
// MT256x256x64_MI16x16x1 / MIWT8_8 / WG32_8_1 kernels use (read off their code object).  Per
// wave and K-tile: 128 MFMAs, 32 fragment reads, 16 LDS-DMA pieces.  Every fragment of a K-tile
// is held in registers (a0/b0: k-step 0, a1/b1: k-step 1, 128 VGPRs), so a buffer is free for
// the tile two ahead as soon as its last fragment read has retired:
//   section 1 (64 MFMAs on a0 x b0): reads of a1/b1 (buffer cur) one per MFMA over the first 16;
//     after MFMA 31 lgkmcnt(0) + barrier (WAR: every wave's reads of cur retired), then the 16
//     DMA pieces of tile t+2 into cur, one per 5 MFMAs;
//   section 2 (64 MFMAs on a1 x b1): the rest of the DMA; after MFMA 47 vmcnt(16) + barrier
//     (RAW: every wave's pieces of tile t+1 landed), then the reads of a0/b0 of tile t+1 (buffer
//     nxt) one per MFMA over the last 16.
// Program order is pinned with sched_barrier(0) after each MFMA step; the compiler inserts the
// counted lgkmcnt waits for the fragment reads, the DMA (inline asm) is counted by hand.

template <typename T, typename OT, int EPI, int DV>
__global__ __launch_bounds__(THREADS4, 1) void gemm_nt4_k(const T* __restrict__ A, long lda,
                                                          const T* __restrict__ B, long ldb, OT* __restrict__ C,
                                                          long ldc, int M, int N, int K, int accumulate, int wide,
                                                          OT* __restrict__ act, int F) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;

  const int nbm = M / TM, nbn = N / TN, nblk = nbm * nbn;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int per_group = GROUP_M * nbn;
  const int grp = wid / per_group;
  const int first_m = grp * GROUP_M;
  const int gm = nbm - first_m < GROUP_M ? nbm - first_m : GROUP_M;
  const int in_g = wid - grp * per_group;
  const int tm = first_m + in_g % gm, tn = in_g / gm;
  const long m0 = (long)tm * TM, n0 = (long)tn * TN;
  const long g0 = (long)tn * 128, u0 = (long)F + (long)tn * 128;

  // ---- staging: wave w moves image rows 64w .. 64w+63 of A and of B, 8 pieces of 8 rows each;
  //      lane l -> row 8p + (l >> 3) of the piece set, physical chunk l & 7 holding logical chunk
  //      (l & 7) ^ ((row >> 1) & 7), which only depends on the piece's parity
  const uint32_t lds0 = lds_u32(smem);
  const long brow0 = EPI == EPI_SWIGLU ? (wave < 2 ? g0 + 64 * wave : u0 + 64 * (wave - 2)) : n0 + 64 * wave;
  const T* Abase = A + (m0 + 64 * wave) * lda;
  const T* Bbase = B + brow0 * ldb;
  const uint32_t ldab = (uint32_t)(lda * sizeof(T)), ldbb = (uint32_t)(ldb * sizeof(T));
  // per-piece lane offsets (row 8p + (l >> 3) of the wave's 64, swizzled chunk) in VGPRs; the
  // tile's base pointer is wave-uniform (SGPRs), so a piece costs one m0 write and the DMA
  uint32_t voA[8], voB[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const uint32_t r = 8u * p + (uint32_t)(lane >> 3), c = 16u * ((lane & 7) ^ ((r >> 1) & 7));
    voA[p] = r * ldab + c;
    voB[p] = r * ldbb + c;
  }
  // piece k of tile t (k < 8: A piece k, k >= 8: B piece k - 8) into buffer buf
  const i32x4 rsA = g4::make_rsrc(Abase), rsB = g4::make_rsrc(Bbase);
  auto dma = [&](int t, int buf, int k) {
    const int p = k & 7;
    const uint32_t d = lds0 + (k >= 8 ? 2 * IMGB : 0) + buf * IMGB + (64 * wave + 8 * p) * ROWB;
    if constexpr (DV == 0) {
      if (k < 8) glds16s(sgpr_ptr(Abase + (long)t * TK), voA[p], d);
      else glds16s(sgpr_ptr(Bbase + (long)t * TK), voB[p], d);
    } else {
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(t * TK * (int)sizeof(T)));
      if (k < 8) g4::bdma16<DV>(rsA, voA[p], so, d);
      else g4::bdma16<DV>(rsB, voB[p], so, d);
    }
  };

  // ---- fragment reads: row (.. + (l & 15)), logical chunk 4s + (l >> 4)
  const int xo0 = ((0 + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4;
  const int xo1 = ((4 + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4;
  // (both buffers of an operand within one 64 KiB window: 4 base VGPRs, the rest immediates)
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

  const int nt = K / TK;  // even, >= 2 (host: K % 128 == 0)
#pragma unroll
  for (int k = 0; k < 16; ++k) dma(0, 0, k);
#pragma unroll
  for (int k = 0; k < 16; ++k) dma(1, 1, k);
  wait_vm<16>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = rdA(0, i, 0), b0[i] = rdB(0, i, 0);

  // One branch-free body for every tile (so hipcc keeps one register assignment and never copies
  // an accumulator between MFMAs, which would read it before the MFMA's result has landed): the
  // pieces "of tile t+2" re-load tile nt-1 when t+2 >= nt (valid memory, into a buffer nothing
  // reads again) and the last tile's "next" fragments are read from a buffer whose contents go
  // unused; every DMA is drained before the epilogue reuses LDS.
  auto tile = [&](int t, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value, nxt = cur ^ 1;
    const int tf = t + 2 < nt ? t + 2 : nt - 1;
    // section 1: a0 x b0; reads of k-step 1 (a1[0], b1[0..7], a1[1..7]) over the first 16 MFMAs
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      const int i = n >> 3, j = n & 7;
      MfA<T>::run(acc[i][j], b0[j], a0[i]);   // swapped: lane holds 4 columns of a row
      if (n == 0) a1[0] = rdA(cur, 0, 1);
      else if (n <= 8) b1[n - 1] = rdB(cur, n - 1, 1);
      else if (n < 16) a1[n - 8] = rdA(cur, n - 8, 1);
      if (n == 31) {   // WAR: every wave's reads of buffer cur retired
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      if (n >= 32 && (n - 32) % 5 == 0) dma(tf, cur, (n - 32) / 5);   // pieces 0..6
      __builtin_amdgcn_sched_barrier(0);
    }
    // section 2: a1 x b1; DMA pieces 7..15; RAW sync for tile t+1; its k-step 0 reads
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      const int i = n >> 3, j = n & 7;
      if (n >= 3 && n <= 43 && (n - 3) % 5 == 0) dma(tf, cur, 7 + (n - 3) / 5);   // pieces 7..15
      if (n == 48) {   // RAW: every wave's pieces of tile t+1 landed (16 of tile t+2 may fly)
        wait_vm<16>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      if (n >= 48) {
        const int r = n - 48;   // a0[0], b0[0..7], a0[1..7]
        if (r == 0) a0[0] = rdA(nxt, 0, 0);
        else if (r <= 8) b0[r - 1] = rdB(nxt, r - 1, 0);
        else a0[r - 8] = rdA(nxt, r - 8, 0);
      }
      MfA<T>::run(acc[i][j], b1[j], a1[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (int t = 0; t < nt; t += 2) {   // nt is even
    tile(t, I0{});
    tile(t + 1, I1{});
  }
  // the last MFMAs' results land before anything reads an accumulator: drain, then pin every
  // accumulator in its AGPR behind the drain (no copy of one can be scheduled above it)
  wait_vm0();
  g4::mfma_drain();
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));

  g4::epilogue4<T, OT, EPI>(acc, smem, wm, wn, lane, C, ldc, m0, n0, g0, u0, accumulate, wide, act, F);
}

// ---- persistent 4-wave schedule (BLLM_GEMM_NT_SCHED=3): the loop of gemm_nt4_k, but one
// workgroup per CU walks output tiles tid, tid + G, ... (the same XCD-contiguous, GROUP_M-deep
// tile order), and the K-tile stream never drains between output tiles: the pieces "of K-tile
// t+2" issued in the last two K-tiles of a tile are K-tiles 0 and 1 of the workgroup's NEXT tile,
// and the fragments read at the end of the last K-tile are that tile's first.  The epilogue
// therefore writes straight from the accumulators (lane: 4 consecutive columns of one row ->
// one 8-B bf16/fp16 or 16-B fp32 store per accumulator) while the next tile's first 64 KiB land
// in LDS, instead of staging through LDS with the pipeline drained.
// SV (BLLM_GEMM_NT4P_SV, A/B): where the WAR barrier, the 16 pieces and the RAW barrier sit in
// the 128-MFMA K-tile.  0: WAR after MFMA 31, pieces every 5 MFMAs from 32, RAW at 112 (reads of
// the next fragments one per MFMA over the last 16); 1: WAR after 23, pieces every 4 from 24,
// RAW at 112; 2: as 1 with RAW at 120 (two reads per MFMA over the last 8); 3: as 0, RAW at 120.
// 4: as 0 with the MFMA order j-major (the B fragment, MFMA src A, fixed over 8 consecutive MFMAs,
// as in hipBLASLt's loop) and the fragment reads ordered to match (b[0], a[0..7], b[1..7]).
// 5: the placement of gfx950 hipBLASLt's MT256x256x64 loop (read off its code object): WAR after
// MFMA 25, pieces every 5 from 26, RAW before MFMA 106, next-fragment reads one per MFMA from there.
template <int SV> struct Sched4 {
  static constexpr bool JMAJ = SV == 4;
  static constexpr int WAR = (SV == 1 || SV == 2) ? 23 : (SV == 5 ? 25 : 31);   // barrier after this MFMA
  static constexpr int D0 = WAR + 1, DS = (SV == 1 || SV == 2) ? 4 : 5;   // first piece, stride
  static constexpr int RAW = SV == 5 ? 106 : ((SV >= 2) ? 120 : 112);     // before this MFMA (of 128)
  // next-tile fragment reads per MFMA from RAW on (1, or 2 when fewer than 16 MFMAs remain)
  static constexpr int RPM = 128 - RAW >= 16 ? 1 : 16 / (128 - RAW);
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
template <typename T, typename OT, int DV, bool ACC, int SV, int EPI = EPI_NONE>
__global__ __launch_bounds__(THREADS4, 1) void gemm_nt4p_k(const T* __restrict__ A, long lda,
                                                           const T* __restrict__ B, long ldb, OT* __restrict__ C,
                                                           long ldc, int M, int N, int K, OT* __restrict__ act = nullptr,
                                                           int F = 0, const float* __restrict__ cosT = nullptr,
                                                           const float* __restrict__ sinT = nullptr, int Tq = 1,
                                                           int nrot = 0, int group_m = GROUP_M,
                                                           const OT* __restrict__ bias = nullptr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int nbm = M / TM, nbn = N / TN, nblk = nbm * nbn, G = gridDim.x;
  const int q8 = nblk >> 3, r8 = nblk & 7, per_group = group_m * nbn;
  auto coords = [&](int tid, long& m0, long& n0) {
    const int xcd = tid & 7;
    const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (tid >> 3);
    const int grp = wid / per_group, first_m = grp * group_m;
    const int gm = nbm - first_m < group_m ? nbm - first_m : group_m;
    const int in_g = wid - grp * per_group;
    m0 = (long)(first_m + in_g % gm) * TM;
    n0 = (long)(in_g / gm) * TN;
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
    g4::bdma16<DV>(k < 8 ? rsA : rsB, k < 8 ? voA[p] : voB[p], soK, d);
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

  using SC = Sched4<SV>;
  // read r (0..15) of a k-step's fragments, in the order the MFMAs consume them
  auto rd16 = [&](s16x8 (&fa)[8], s16x8 (&fb)[8], int buf, int s, int r) {
    if constexpr (SC::JMAJ) {
      if (r == 0) fb[0] = rdB(buf, 0, s);
      else if (r <= 8) fa[r - 1] = rdA(buf, r - 1, s);
      else fb[r - 8] = rdB(buf, r - 8, s);
    } else {
      if (r == 0) fa[0] = rdA(buf, 0, s);
      else if (r <= 8) fb[r - 1] = rdB(buf, r - 1, s);
      else fa[r - 8] = rdA(buf, r - 8, s);
    }
  };
  auto ktile = [&](int t, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value, nxt = cur ^ 1;
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      const int i = SC::JMAJ ? (n & 7) : (n >> 3), j = SC::JMAJ ? (n >> 3) : (n & 7);
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
      const int i = SC::JMAJ ? (n & 7) : (n >> 3), j = SC::JMAJ ? (n >> 3) : (n & 7);
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
            gb[e] = from_f<OT>(0.5f * x * (1.f + erff(x * 0.70710678118654752f)));
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
            w[e] = from_f<OT>(a / (1.f + __expf(-a)) * b);
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

// BLLM_GEMM_NT_SCHED (read per launch, so one process can A/B): 0 = one barrier per K-tile
// (gemm_nt_k), 1 = ping-pong wave rows (gemm_nt_pp_k), 2 = 4 waves of 128 x 128 (gemm_nt4_k)
inline int nt_sched() {
  const char* e = getenv("BLLM_GEMM_NT_SCHED");
  return e ? atoi(e) : 0;
}

template <typename T, typename OT>
void launch_swiglu4p(const void* a, long lda, const void* b, long ldb, void* c, long ldc, int M, int N, int K,
                     void* act, int F, hipStream_t s) {
    static int ncu_s = 0;
  if (!ncu_s) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    ncu_s = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    ncu_s = ncu_s < 8 ? 8 : ncu_s / 8 * 8;
  }
  static const bool at_s = hipFuncSetAttribute((const void*)gemm_nt4p_k<T, OT, 1, false, 0, EPI_SWIGLU>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
  (void)at_s;
  const int nblk = (M / TM) * (N / TN);
  const int grid = nblk < ncu_s ? nblk : ncu_s;
  hipLaunchKernelGGL((gemm_nt4p_k<T, OT, 1, false, 0, EPI_SWIGLU>), dim3(grid), dim3(THREADS4), LDS_BYTES, s,
                     (const T*)a, lda, (const T*)b, ldb, (OT*)c, ldc, M, N, K, (OT*)act, F);
}

template <typename T, typename OT, int EPI = EPI_NONE>
void launch(const void* a, long lda, const void* b, long ldb, void* c, long ldc, int M, int N, int K, bool accumulate,
            hipStream_t s, void* act = nullptr, int F = 0, int sched = -1) {
  static const bool attr = hipFuncSetAttribute((const void*)gemm_nt_k<T, OT, EPI>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess &&
                           hipFuncSetAttribute((const void*)gemm_nt_pp_k<T, OT, EPI>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess &&
                           hipFuncSetAttribute((const void*)gemm_nt4_k<T, OT, EPI, 0>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess &&
                           hipFuncSetAttribute((const void*)gemm_nt4_k<T, OT, EPI, 1>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess &&
                           hipFuncSetAttribute((const void*)gemm_nt4_k<T, OT, EPI, 2>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess &&
                           hipFuncSetAttribute((const void*)gemm_nt4_k<T, OT, EPI, 3>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
  (void)attr;
  const bool wide = reinterpret_cast<uintptr_t>(c) % 16 == 0 && (ldc * (long)sizeof(OT)) % 16 == 0;
  const int sc = sched < 0 ? nt_sched() : sched;
  const bool vec3 = sizeof(OT) == 2 ? (reinterpret_cast<uintptr_t>(c) % 8 == 0 && (ldc * (long)sizeof(OT)) % 8 == 0)
                                    : (reinterpret_cast<uintptr_t>(c) % 16 == 0 && (ldc * (long)sizeof(OT)) % 16 == 0);
  if constexpr (EPI == EPI_SWIGLU && sizeof(OT) == 2) {
    if (sc == 3 && vec3 && F % 4 == 0) {
      launch_swiglu4p<T, OT>(a, lda, b, ldb, c, ldc, M, N, K, act, F, s);
      return;
    }
  }
  if (sc == 3 && EPI == EPI_NONE && vec3) {
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      hipDeviceProp_t prop;
      ncu = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
      ncu = ncu < 8 ? 8 : ncu / 8 * 8;
    }
    const int nblk = (M / TM) * (N / TN);
    const int grid = nblk < ncu ? nblk : ncu;
    const char* ev = getenv("BLLM_GEMM_NT4P_SV");
    const int sv = ev && *ev ? atoi(ev) : 0;
    const char* eg = getenv("BLLM_GEMM_NT4P_GM");   // tile-group depth (A/B); default GROUP_M
    // 4 measured 0.3-12 % faster than 8 (16, 32 slower) on the Llama-3-8B / GPT2-774M shapes
    // (profiles/r3/gemm_nt4p_sv4_gm.jsonl)
    const int gmz = eg && atoi(eg) > 0 ? atoi(eg) : 4;
#define BLLM_NT4P(ACCv, SVv, DVv)                                                                                       \
  do {                                                                                                                  \
    static const bool at_ = hipFuncSetAttribute((const void*)gemm_nt4p_k<T, OT, DVv, ACCv, SVv>,                        \
                                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess; \
    (void)at_;                                                                                                          \
    hipLaunchKernelGGL((gemm_nt4p_k<T, OT, DVv, ACCv, SVv>), dim3(grid), dim3(THREADS4), LDS_BYTES, s, (const T*)a,   \
                       lda, (const T*)b, ldb, (OT*)c, ldc, M, N, K, (OT*)nullptr, 0, nullptr, nullptr, 1, 0, gmz);  \
  } while (0)
    // sv 5 / 6: schedule 0 with the pieces issued sc0 sc1 / nt (cache-policy A/B)
    if (accumulate) {
      BLLM_NT4P(true, 0, 1);
    } else if (sv == 1) {
      BLLM_NT4P(false, 1, 1);
    } else if (sv == 2) {
      BLLM_NT4P(false, 2, 1);
    } else if (sv == 3) {
      BLLM_NT4P(false, 3, 1);
    } else if (sv == 4) {
      BLLM_NT4P(false, 4, 1);
    } else if (sv == 7) {
      BLLM_NT4P(false, 5, 1);
    } else if (sv == 5) {
      BLLM_NT4P(false, 0, 2);
    } else if (sv == 6) {
      BLLM_NT4P(false, 0, 3);
    } else {
      BLLM_NT4P(false, 0, 1);
    }
#undef BLLM_NT4P
  } else if (sc == 2 || sc == 3) {
    const char* e = getenv("BLLM_GEMM_NT4_DMA");
    const int dv = e && *e ? atoi(e) : 0;
#define BLLM_NT4(DVv)                                                                                                  \
  hipLaunchKernelGGL((gemm_nt4_k<T, OT, EPI, DVv>), dim3((M / TM) * (N / TN)), dim3(THREADS4), LDS_BYTES, s,         \
                     (const T*)a, lda, (const T*)b, ldb, (OT*)c, ldc, M, N, K, (int)accumulate, (int)wide, (OT*)act, F)
    if (dv == 1) BLLM_NT4(1);
    else if (dv == 2) BLLM_NT4(2);
    else if (dv == 3) BLLM_NT4(3);
    else BLLM_NT4(0);
#undef BLLM_NT4
  } else if (sc == 1)
    hipLaunchKernelGGL((gemm_nt_pp_k<T, OT, EPI>), dim3((M / TM) * (N / TN)), dim3(THREADS), LDS_BYTES, s,
                       (const T*)a, lda, (const T*)b, ldb, (OT*)c, ldc, M, N, K, (int)accumulate, (int)wide, (OT*)act, F);
  else
    hipLaunchKernelGGL((gemm_nt_k<T, OT, EPI>), dim3((M / TM) * (N / TN)), dim3(THREADS), LDS_BYTES, s, (const T*)a,
                       lda, (const T*)b, ldb, (OT*)c, ldc, M, N, K, (int)accumulate, (int)wide, (OT*)act, F);
}

}  // namespace

bool gemm_nt_rope_supported(int M, int N, int K, long lda, long ldb, long ldc, int hd) {
  return hd == 128 && M > 0 && N > 0 && M % TM == 0 && N % TN == 0 && K % (2 * TK) == 0 && ldc % 4 == 0 &&
         (long)TM * lda * 2 < (1L << 31) && (long)TN * ldb * 2 < (1L << 31);
}

void gemm_nt_rope(DType dt, const void* a, long lda, const void* w, long ldw, void* c, long ldc, int M, int N, int K,
                  const float* cosT, const float* sinT, int Tq, int nrot, hipStream_t s) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    ncu = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    ncu = ncu < 8 ? 8 : ncu / 8 * 8;
  }
  const int nblk = (M / TM) * (N / TN);
  const int grid = nblk < ncu ? nblk : ncu;
#define BLLM_ROPE4P(TT)                                                                                                \
  do {                                                                                                                 \
    static const bool at_ = hipFuncSetAttribute((const void*)gemm_nt4p_k<TT, TT, 1, false, 0, EPI_ROPE>,              \
                                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess; \
    (void)at_;                                                                                                         \
    hipLaunchKernelGGL((gemm_nt4p_k<TT, TT, 1, false, 0, EPI_ROPE>), dim3(grid), dim3(THREADS4), LDS_BYTES, s,         \
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
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    ncu = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    ncu = ncu < 8 ? 8 : ncu / 8 * 8;
  }
  const int nblk = (M / TM) * (N / TN);
  const int grid = nblk < ncu ? nblk : ncu;
#define BLLM_GELU4P(TT)                                                                                                \
  do {                                                                                                                 \
    static const bool at_ = hipFuncSetAttribute((const void*)gemm_nt4p_k<TT, TT, 1, false, 0, EPI_BIAS_GELU>,         \
                                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess; \
    (void)at_;                                                                                                         \
    hipLaunchKernelGGL((gemm_nt4p_k<TT, TT, 1, false, 0, EPI_BIAS_GELU>), dim3(grid), dim3(THREADS4), LDS_BYTES, s,    \
                       (const TT*)a, lda, (const TT*)w, ldw, (TT*)f, ldc, M, N, K, (TT*)g, 0, nullptr, nullptr, 1, 0, \
                       4, (const TT*)bias);                                                                            \
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
              int K, bool accumulate, hipStream_t s, int sched) {
  BLLM_DISPATCH(odt, OT, {
    if (dt == DType::BF16) launch<bf16_t, OT>(a, lda, b, ldb, c, ldc, M, N, K, accumulate, s, nullptr, 0, sched);
    else launch<f16_t, OT>(a, lda, b, ldb, c, ldc, M, N, K, accumulate, s, nullptr, 0, sched);
  });
}

bool gemm_nt_swiglu_supported(int M, int F, int K, long lda, long ldb, long ldgu) {
  return F > 0 && F % 128 == 0 && gemm_nt2_supported(M, 2 * F, K, lda, ldb) && ldgu % 8 == 0;
}

void gemm_nt_swiglu(DType dt, const void* a, long lda, const void* w, long ldw, void* gu, long ldgu, void* act, int M,
                    int F, int K, hipStream_t s) {
  // the persistent 4-wave schedule unless BLLM_GEMM_NT_SCHED picks another one (A/B)
  const int sc = getenv("BLLM_GEMM_NT_SCHED") ? -1 : 3;
  if (dt == DType::BF16) launch<bf16_t, bf16_t, EPI_SWIGLU>(a, lda, w, ldw, gu, ldgu, M, 2 * F, K, false, s, act, F, sc);
  else launch<f16_t, f16_t, EPI_SWIGLU>(a, lda, w, ldw, gu, ldgu, M, 2 * F, K, false, s, act, F, sc);
}

}  // namespace bllm
