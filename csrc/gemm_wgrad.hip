// Weight-gradient GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x32_{bf16,f16}).
//
//   C[M, N] (+)= A^T . B      A = [K, M] row-major (lda), B = [K, N] row-major (ldb)
//
// This is the layout of every dW of a Linear: dW[out, in] = dY^T . X with dY [tokens, out] and
// X [tokens, in] — the reduction dimension (tokens) is the OUTER (strided) dimension of both
// operands, so neither is K-contiguous.  hipBLASLt runs this family at 1.0-1.16 PF on the
// Llama-3-8B projections vs 1.5 PF for the forward layout (profiles/r1_llama3_8b_1gpu_v3.md;
// TunableOp over all hipBLASLt/rocBLAS solutions does not close the gap).  Here the operands are
// staged exactly as they sit in memory and the transpose is done by the LDS read instead of a
// copy:
//
//  * tile 256 x 256 per workgroup, 8 waves = 2 (M) x 4 (N), 128 x 64 outputs per wave
//    (acc[8][4]), two waves per SIMD; one 32-deep k-step per LDS ring slot;
//  * a ring of 4 slots (A [32 k][256 m] + B [32 k][256 n] images, 16 KiB each, 128 KiB total)
//    filled by LDS-DMA (global_load_lds_dwordx4) 3 slots ahead of the MFMAs; one raw s_barrier
//    per slot, counted vmcnt (never drained to 0 inside the loop);
//  * fragments are read with ds_read_b64_tr_b16 (a 16-lane group gets 4 k-rows x 16 columns
//    delivered column-major = 4 k-values of one m/n column per lane); two reads give the 8
//    k-values of a 16x16x32 A or B fragment;
//  * bank conflicts: a 32-lane half-wave reads 8 k-rows x 32 B at the same columns; the image
//    XOR-permutes 16-B chunks within each 512-B k-row by f(r) = 2*((r&3) | ((r>>3)&1)<<2), which
//    puts the 8 rows on 8 distinct 32-B bank groups (conflict-free).  The DMA writes LDS
//    lane-linearly, so the permutation is applied to the per-lane GLOBAL source address (a
//    permutation of 16-B chunks inside one 512-B row: the loads stay fully coalesced);
//  * blockIdx.x -> tile: XCD-aware (each XCD gets a contiguous range of tiles, bijective for
//    any count), grouped 8 tile-rows deep so the tiles an XCD runs at once share A and B
//    panels in its L2;
//  * blockIdx.y = split-K index (few-tile GEMMs): split s reduces its own 128-aligned token
//    range into fp32 partial s of C (c_split elements apart), summed afterwards in a fixed
//    order — deterministic either way (each output element has one owner per split).
//
//  * epilogue staged through LDS: the 256 x 256 fp32 tile is written into the (then idle) LDS
//    ring in two 128-row passes and leaves as 16-B row-contiguous global stores (and 16-B loads
//    when accumulating) instead of 128 scattered 2-/4-byte stores per lane.
//
// Two schedules (the others -- fragments read after each barrier, DMA by all 8 waves,
// 32x32x16 MFMAs, a persistent variant of wgrad4_k -- measured slower and were deleted;
// profiles/r2_kernel_experiments.md, profiles/r3/kernel_experiments.md):
//   wgrad_gemm_k  8 waves of 128 x 64, next slot's fragments read under the current slot's
//                 MFMAs, LDS-DMA issued by waves 0-3 only -- deep split-K (S >= 8: few, short
//                 tiles) and the K-contiguous-A dX kernel (gemm_nn);
//   wgrad4_k      4 waves (one per SIMD) of 128 x 128 (below) -- every other weight gradient.
#include <stdlib.h>

#include <type_traits>

#include "api.h"
#include "gemm4.h"

namespace bllm {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  static __device__ __forceinline__ f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
  static __device__ __forceinline__ f32x16 run(s16x8 a, s16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
};
template <> struct Mfma<f16_t> {
  static __device__ __forceinline__ f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
  }
  static __device__ __forceinline__ f32x16 run(s16x8 a, s16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
  }
};

constexpr int BM = 256, BN = 256, BK = 32;  // BK = one MFMA k-step per ring slot
constexpr int NSLOT = 4;
constexpr int KCH = NSLOT * BK;             // K granule (one trip of the unrolled ring)
constexpr int ROWB = 512;                   // bytes of one k-row of a 256-wide image
constexpr int SLOTB = BK * ROWB;            // 16 KiB
constexpr int B_BASE = NSLOT * SLOTB;       // A slots [0, 64 KiB), B slots [64, 128 KiB)
constexpr int LDS_BYTES = 2 * NSLOT * SLOTB;
constexpr int GROUP_M = 8;

// wave layout / schedule of wgrad_gemm_k
struct Geo {
  static constexpr int NW = 8;                         // waves per workgroup
  static constexpr int THREADS = NW * 64;
  static constexpr int WAVES_N = 4;                    // waves along N (2 along M)
  static constexpr int FN = BN / WAVES_N / 16;         // 16-wide n fragments per wave
  // only waves 0-3 (one per SIMD) issue the slot's LDS-DMA, so each SIMD's other wave (4-7) goes
  // straight from the barrier to its MFMAs and keeps the matrix pipe busy while its partner
  // spends ~60 issue cycles per piece (1.02-1.13x splitting the pieces over all 8)
  static constexpr int LOADERS = 4;
  static constexpr int DJ = (SLOTB / 1024) / LOADERS;  // LDS-DMA pieces per operand per slot per loader
  static constexpr int PER_STAGE = 2 * DJ;             // vmcnt units one staged slot adds (loaders)
};

__device__ __forceinline__ int swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

__device__ __forceinline__ s16x8 frag(const char* p) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * ROWB));
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// AK = false: A is [K, M] row-major (token-major dY of a weight gradient; transposed LDS reads).
// AK = true:  A is [M, K] row-major (K-contiguous, e.g. dY of an input gradient dX = dY W):
//             A images are [256 m][32 k] rows of 64 B, 16-B chunk c of row r stored at
//             c ^ fA((r >> 2) & 3) with fA = {0, 2, 3, 1} (every 16-lane ds_read_b128 group then
//             covers 16 distinct bank quads), fragments read with ds_read_b128.
__device__ __forceinline__ int fA(int q) { return (0x78 >> (2 * q)) & 3; }

template <typename T, typename OT, bool AK = false>
__global__ __launch_bounds__(Geo::THREADS) void wgrad_gemm_k(const T* __restrict__ A, long lda,
                                                                  const T* __restrict__ B, long ldb,
                                                                  OT* __restrict__ C, long ldc, long c_split,
                                                                  int M, int N, int K, int accumulate, int wide) {
  using G = Geo;
  constexpr int FN = G::FN, DJ = G::DJ, PS = G::PER_STAGE;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;

  // ---- tile id: XCD-contiguous (bijective), then GROUP_M-deep column-major groups
  const int nbm = M / BM, nbn = N / BN, nblk = nbm * nbn;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int per_group = GROUP_M * nbn;
  const int grp = wid / per_group;
  const int first_m = grp * GROUP_M;
  const int gm = nbm - first_m < GROUP_M ? nbm - first_m : GROUP_M;
  const int in_g = wid - grp * per_group;
  const int tm = first_m + in_g % gm, tn = in_g / gm;
  const long m0 = (long)tm * BM, n0 = (long)tn * BN;

  // ---- this split's token range (128-aligned)
  const int S = gridDim.y, sp = blockIdx.y, nch = K / KCH;
  const int c_lo = (int)((long)nch * sp / S), c_hi = (int)((long)nch * (sp + 1) / S);
  const int nk = (c_hi - c_lo) * NSLOT;  // >= NSLOT (host: S <= K / KCH)

  // ---- staging: lane-linear LDS rows, XOR-permuted global chunks (loop-invariant offsets);
  //      one piece (wave-instruction) moves 2 k-rows (1 KiB) of one operand
  uint32_t voffA[DJ], voffB[DJ];
#pragma unroll
  for (int j = 0; j < DJ; ++j) {
    const int r = (wave * DJ + j) * 2 + (lane >> 5), c = (lane & 31) ^ swz(r);
    voffB[j] = (uint32_t)((r * ldb + 8 * c) * (long)sizeof(T));
    if constexpr (AK) {  // piece = 16 m-rows x 64 B; lane -> row l/4, physical chunk l%4
      const int ra = (wave * DJ + j) * 16 + (lane >> 2), ca = (lane & 3) ^ fA((ra >> 2) & 3);
      voffA[j] = (uint32_t)((ra * lda + 8 * ca) * (long)sizeof(T));
    } else {
      voffA[j] = (uint32_t)((r * lda + 8 * c) * (long)sizeof(T));
    }
  }
  const uint32_t lds0 = lds_u32(smem);
  const T* Abase = AK ? A + m0 * lda + (long)c_lo * KCH : A + (long)c_lo * KCH * lda + m0;
  const T* Bbase = B + (long)c_lo * KCH * ldb + n0;
  // piece q of a stage: q even = A piece q/2, q odd = B piece q/2 (issue order A0 B0 A1 B1 ..)
  auto piece = [&](const void* a, const void* b, int q, int slot) {
    const int j = q >> 1;
    if (q & 1) glds16s(b, voffB[j], lds0 + B_BASE + slot * SLOTB + (wave * DJ + j) * 1024);
    else glds16s(a, voffA[j], lds0 + slot * SLOTB + (wave * DJ + j) * 1024);
  };
  auto stage = [&](int kt, int slot) {
    if (wave >= G::LOADERS) return;  // wave-uniform (readfirstlane'd)
    const void* a = sgpr_ptr(Abase + (AK ? (long)kt * BK : (long)kt * BK * lda));
    const void* b = sgpr_ptr(Bbase + (long)kt * BK * ldb);
#pragma unroll
    for (int q = 0; q < PS; ++q) piece(a, b, q, slot);
  };

  // ---- fragment read offsets: lane (g, q, p) reads k-row 8g + q (+4), columns 4p..4p+3
  const int g = lane >> 4, qq = (lane & 15) >> 2, p = lane & 3;
  const int f = 2 * (qq | ((g & 1) << 2));  // == swz(8g + qq + 4h) for h = 0, 1
  const int wm = wave / G::WAVES_N, wn = wave % G::WAVES_N;
  const int rowb = (8 * g + qq) * ROWB + (p & 1) * 8 + (p >> 1) * 16;
  int aoff[8], boff[FN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    aoff[i] = AK ? (wm * 128 + 16 * i + (lane & 15)) * 64 + (((lane >> 4) ^ fA((lane & 15) >> 2)) << 4)
                 : rowb + (wm * 16 + ((2 * i) ^ f)) * 16;
  // A fragment: 8 k-values of one m row (row read) or of one m column (two transposed reads)
  auto fragA = [&](const char* p) -> s16x8 {
    if constexpr (AK) return *(const __attribute__((address_space(3))) s16x8*)(p);
    else return frag(p);
  };
#pragma unroll
  for (int j = 0; j < FN; ++j)
    boff[j] = B_BASE + rowb + ((wn * 2 * FN + 2 * j) ^ f) * 16;
  // B fragment: 8 k-values of one n column (two transposed reads)
  auto fragB = [&](const char* p) -> s16x8 { return frag(p); };

  f32x4 acc[8][FN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{};

  {
    // Fragments of slot kt+1 are read into the second register set WHILE slot kt's MFMAs
    // run, so no wave waits on LDS latency after a barrier: the MFMA pipe stays fed across it.
    // Ring: DMA of k-slot kt+4 refills LDS slot kt as soon as every wave holds slot kt in VGPRs.
    struct Frags { s16x8 a[8], b[FN]; };
    auto load = [&](Frags& F, int slot) {
      const char* base = smem + slot * SLOTB;
#pragma unroll
      for (int j = 0; j < FN; ++j) F.b[j] = fragB(base + boff[j]);
#pragma unroll
      for (int i = 0; i < 8; ++i) F.a[i] = fragA(base + aoff[i]);
    };
    // G.b first, then G.a[i] just before F.a[i]'s MFMAs: F.a[i] dies as G.a[i] arrives, so the
    // two sets cost 2 x FN B-fragments + 9 A-fragments of VGPRs, not 2 x (8 + FN).  The loop
    // body is branch-free (the final trip is peeled) so hipcc's lgkmcnt counting stays exact.
    auto it = [&](auto wait_n, auto do_stage, auto last, int kt, Frags& F, Frags& Gn) {
      constexpr int WAITN = decltype(wait_n)::value;
      constexpr bool STAGE = decltype(do_stage)::value, LAST = decltype(last)::value;
      const char* nxt = smem + ((kt + 1) & (NSLOT - 1)) * SLOTB;
      if constexpr (!LAST) {
        vm_wait<WAITN>();  // DMA kt+1 landed (later slots may still fly)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // F (= LDS slot kt) is in VGPRs
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if constexpr (STAGE) stage(kt + 4, kt & (NSLOT - 1));
#pragma unroll
        for (int j = 0; j < FN; ++j) Gn.b[j] = fragB(nxt + boff[j]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (!LAST) Gn.a[i] = fragA(nxt + aoff[i]);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = Mfma<T>::run(F.a[i], F.b[j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    };
    using W2 = std::integral_constant<int, 2 * PS>;  // 2 slots still in flight behind kt+1
    using W1 = std::integral_constant<int, PS>;
    using W0 = std::integral_constant<int, 0>;
    using Y = std::true_type;
    using Nn = std::false_type;
    stage(0, 0);
    stage(1, 1);
    stage(2, 2);
    stage(3, 3);
    vm_wait<3 * PS>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    Frags F0, F1;
    load(F0, 0);
    int kt = 0;
    for (; kt < nk - NSLOT; kt += NSLOT) {
      it(W2{}, Y{}, Nn{}, kt + 0, F0, F1);
      it(W2{}, Y{}, Nn{}, kt + 1, F1, F0);
      it(W2{}, Y{}, Nn{}, kt + 2, F0, F1);
      it(W2{}, Y{}, Nn{}, kt + 3, F1, F0);
    }
    it(W2{}, Nn{}, Nn{}, kt + 0, F0, F1);
    it(W1{}, Nn{}, Nn{}, kt + 1, F1, F0);
    it(W0{}, Nn{}, Nn{}, kt + 2, F0, F1);
    it(W0{}, Nn{}, Y{}, kt + 3, F1, F0);
  }

  // ---- epilogue: lane holds C[16i + 4(l>>4) + e][16j + (l&15)] of the wave's 128 x 64 block
  OT* cbase = C + sp * c_split + m0 * ldc + n0;
  if (wide) {
    // Through LDS: fp32 rows of 1 KiB (16-B chunk index XOR (row & 7): the two rows a 32-lane
    // half writes land on disjoint banks), pass p = the 128 rows of the waves with wm == p; then
    // every thread moves whole 16-B global chunks (4 fp32 or 8 bf16/fp16 elements).
    constexpr int RB = BN * 4;
    constexpr int EPT = 16 / (int)sizeof(OT);  // elements per 16-B global access
    constexpr int NCH = EPT / 4;               // fp32 LDS chunks per access
    constexpr int IPR = BN / EPT;              // accesses per row
    constexpr int TRIPS = 128 * IPR / G::THREADS;
    struct alignas(16) V16 { OT e[EPT]; };
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every LDS read of the ring is done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (wm == pass) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              const int lr = 16 * i + 4 * (lane >> 4) + e, col = wn * 16 * FN + 16 * j + (lane & 15);
              *(float*)(smem + lr * RB + ((((col >> 2) ^ (lr & 7)) << 4) | ((col & 3) << 2))) = acc[i][j][e];
            }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int t = 0; t < TRIPS; ++t) {
        const int q = (int)threadIdx.x + t * G::THREADS;
        const int lr = q / IPR, it = q % IPR;
        float v[EPT];
#pragma unroll
        for (int h = 0; h < NCH; ++h) {
          const f32x4 x = *(const f32x4*)(smem + lr * RB + (((it * NCH + h) ^ (lr & 7)) << 4));
#pragma unroll
          for (int k = 0; k < 4; ++k) v[4 * h + k] = x[k];
        }
        V16* o = (V16*)(cbase + (long)(pass * 128 + lr) * ldc + it * EPT);
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
      if (pass == 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // pass-0 reads done before pass 1 writes
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    }
    return;
  }
  // (unaligned output: element stores; the accumulate test is hoisted out of the element loops —
  //  a per-element select makes hipcc branch around every load and wait for each separately)
  OT* c = cbase + (wm * 128 + 4 * (lane >> 4)) * ldc + wn * 16 * FN + (lane & 15);
  if (accumulate) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          OT* o = c + (long)(16 * i + e) * ldc + 16 * j;
          *o = from_f<OT>(to_f(*o) + acc[i][j][e]);
        }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < FN; ++j) c[(long)(16 * i + e) * ldc + 16 * j] = from_f<OT>(acc[i][j][e]);
  }
}

// ---- Variant 4: one wave per SIMD, 128 x 128 outputs per wave (the structure of
// csrc/gemm_nt.hip's 4-wave schedule and of gfx950 hipBLASLt's MT256x256x64 kernels) on this
// kernel's operand layout.  A K-tile is 64 tokens = two 32-row ring slots per operand (LDS slots
// 2b, 2b+1 of buffer b; same images, swizzle and transposed fragment reads as wgrad_gemm_k);
// every fragment of a K-tile sits in VGPRs (a0/b0 k-step 0, a1/b1 k-step 1), the MFMAs keep their
// accumulators in place in AGPRs (g4::MfA), operands swapped so a lane holds 4 consecutive
// columns of a row (g4::epilogue4).  Per wave and K-tile: 128 MFMAs, 64 ds_read_b64_tr_b16,
// 16 LDS-DMA pieces (wave w moves token rows 16w .. 16w+15 of both operands):
//   section 1 (a0 x b0): reads of a1/b1 over the first 16 MFMAs; after MFMA 31 lgkmcnt(0) +
//     barrier (WAR on buffer cur), then the pieces of tile t+2 into cur, one per 5 MFMAs;
//   section 2 (a1 x b1): the rest of the pieces; after MFMA 47 vmcnt(16) + barrier (RAW for tile
//     t+1), then the reads of a0/b0 of tile t+1 over the last 16 MFMAs.
// The body is branch-free for every tile (past the end the pieces re-load the last tile into a
// buffer nothing reads again).  Pieces are buffer_load ... lds on a per-K-tile descriptor.
// tile maps (``map``, set_gemm_tile_maps): 0 = XCD-contiguous over GROUP_M-deep column-major
// groups (each XCD an M-band), 1 = plain bid order, 2 = the same over the transposed grid (each XCD
// an N-band); ``group_m`` = group depth
// grouped tile order -> (tm, tn): GROUP_M-deep column-major groups (map 2: over the transposed
// grid); shared by wgrad4_k and the split-tail reduction
__device__ __forceinline__ void wg_tile(int wid, int nbm, int nbn, int map, int group_m, int& tm, int& tn) {
  const bool trg = map == 2;
  const int gmaj = trg ? nbn : nbm, gmin = trg ? nbm : nbn;
  const int per_group = group_m * gmin;
  const int grp = wid / per_group;
  const int first_m = grp * group_m;
  const int gm = gmaj - first_m < group_m ? gmaj - first_m : group_m;
  const int in_g = wid - grp * per_group;
  const int ta = first_m + in_g % gm, tb = in_g / gm;
  tm = trg ? tb : ta;
  tn = trg ? ta : tb;
}

// tile0 / ntile: this launch covers tiles [tile0, tile0 + ntile) of the grouped order (the
// XCD-contiguous deal is over those ntile).  compact (split tails): split sp of the launch's local
// tile t writes its fp32 256 x 256 partial at C + ((sp * ntile + t) * 256 * 256), row stride 256.
template <typename T, typename OT>
__global__ __launch_bounds__(g4::THREADS4, 1) void wgrad4_k(const T* __restrict__ A, long lda,
                                                            const T* __restrict__ B, long ldb, OT* __restrict__ C,
                                                            long ldc, long c_split, int M, int N, int K,
                                                            int accumulate, int wide, int map = 0,
                                                            int group_m = GROUP_M, int tile0 = 0, int ntile = -1,
                                                            int compact = 0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;

  const int nbm = M / BM, nbn = N / BN;
  const int cnt = ntile < 0 ? nbm * nbn : ntile;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = cnt >> 3, r8 = cnt & 7;
  const int local = map == 1 ? bid : (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int wid = tile0 + local;
  int tm, tn;
  wg_tile(wid, nbm, nbn, map, group_m, tm, tn);
  const long m0 = (long)tm * BM, n0 = (long)tn * BN;

  const int S = gridDim.y, sp = blockIdx.y, nch = K / KCH;
  const int c_lo = (int)((long)nch * sp / S), c_hi = (int)((long)nch * (sp + 1) / S);
  const int nt = (c_hi - c_lo) * (KCH / 64);   // 64-deep K-tiles, even

  // ---- staging: piece p of wave w = token rows kr, kr+1 (kr = 16w + 2p) of the K-tile; lane l
  //      -> row kr + (l >> 5), physical chunk l & 31 holding logical chunk (l & 31) ^ swz(row & 31)
  uint32_t voA[8], voB[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int kr = 16 * wave + 2 * p + (lane >> 5), c = (lane & 31) ^ swz(kr & 31);
    voA[p] = (uint32_t)((kr * lda + 8 * c) * (long)sizeof(T));
    voB[p] = (uint32_t)((kr * ldb + 8 * c) * (long)sizeof(T));
  }
  const uint32_t lds0 = lds_u32(smem);
  const T* Abase = A + (long)c_lo * KCH * lda + m0;
  const T* Bbase = B + (long)c_lo * KCH * ldb + n0;
  // piece k (< 8: A piece k, else B piece k - 8) of tile t into buffer buf (slots 2buf, 2buf+1)
  auto dma = [&](int t, int buf, int k) {
    const int p = k & 7, kr = 16 * wave + 2 * p;
    const uint32_t d = lds0 + (k >= 8 ? B_BASE : 0) + (2 * buf + (kr >> 5)) * SLOTB + (kr & 31) * ROWB;
    const T* base = k < 8 ? Abase + (long)t * 64 * lda : Bbase + (long)t * 64 * ldb;
    g4::bdma16<1>(g4::make_rsrc(base), k < 8 ? voA[p] : voB[p], 0u, d);
  };

  // ---- fragment offsets (those of wgrad_gemm_k with 128 columns per wave on both operands)
  const int g = lane >> 4, qq = (lane & 15) >> 2, p4 = lane & 3;
  const int f = 2 * (qq | ((g & 1) << 2));
  const int rowb = (8 * g + qq) * ROWB + (p4 & 1) * 8 + (p4 >> 1) * 16;
  const char* pa = smem + rowb + (wm * 16) * 16;
  const char* pb = smem + B_BASE + rowb + (wn * 16) * 16;
  // i-th 16-column fragment of slot sl: column chunk (2i) ^ f past the wave's base (f < 16, even)
  auto rdA = [&](int sl, int i) -> g4::s16x8 { return frag(pa + sl * SLOTB + ((2 * i) ^ f) * 16); };
  auto rdB = [&](int sl, int j) -> g4::s16x8 { return frag(pb + sl * SLOTB + ((2 * j) ^ f) * 16); };

  g4::f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = g4::f32x4{};
  g4::s16x8 a0[8], b0[8], a1[8], b1[8];

#pragma unroll
  for (int k = 0; k < 16; ++k) dma(0, 0, k);
#pragma unroll
  for (int k = 0; k < 16; ++k) dma(1, 1, k);
  vm_wait<16>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = rdA(0, i), b0[i] = rdB(0, i);

  auto tile = [&](int t, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value, nxt = cur ^ 1;
    const int tf = t + 2 < nt ? t + 2 : nt - 1;
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      const int i = n >> 3, j = n & 7;
      g4::MfA<T>::run(acc[i][j], b0[j], a0[i]);
      if (n == 0) a1[0] = rdA(2 * cur + 1, 0);
      else if (n <= 8) b1[n - 1] = rdB(2 * cur + 1, n - 1);
      else if (n < 16) a1[n - 8] = rdA(2 * cur + 1, n - 8);
      if (n == 31) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      if (n >= 32 && (n - 32) % 5 == 0) dma(tf, cur, (n - 32) / 5);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      const int i = n >> 3, j = n & 7;
      if (n >= 3 && n <= 43 && (n - 3) % 5 == 0) dma(tf, cur, 7 + (n - 3) / 5);
      if (n == 48) {
        vm_wait<16>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      if (n >= 48) {
        const int r = n - 48;
        if (r == 0) a0[0] = rdA(2 * nxt, 0);
        else if (r <= 8) b0[r - 1] = rdB(2 * nxt, r - 1);
        else a0[r - 8] = rdA(2 * nxt, r - 8);
      }
      g4::MfA<T>::run(acc[i][j], b1[j], a1[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (int t = 0; t < nt; t += 2) {
    tile(t, I0{});
    tile(t + 1, I1{});
  }
  vm_wait<0>();
  g4::mfma_drain();
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  if (compact)
    g4::epilogue4<T, OT, g4::EPI_NONE>(acc, smem, wm, wn, lane, C + ((long)sp * cnt + local) * BM * BN, BN, 0, 0, 0,
                                       0, 0, 1, (OT*)nullptr, 0);
  else
    g4::epilogue4<T, OT, g4::EPI_NONE>(acc, smem, wm, wn, lane, C + sp * c_split, ldc, m0, n0, 0, 0, accumulate, wide,
                                       (OT*)nullptr, 0);
}

// c[tile] (+)= sum_s part[s][t] over the split-tail tiles t < ntile (fixed order: deterministic);
// 8 consecutive outputs per thread
template <typename OT>
__global__ __launch_bounds__(256) void wg_tail_sum_k(const float* __restrict__ part, OT* __restrict__ C, long ldc,
                                                     int M, int N, int tile0, int ntile, int S, int map, int group_m,
                                                     int accumulate) {
  const long per_tile = (long)BM * BN / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < per_tile * ntile; i += (long)gridDim.x * 256) {
    const int t = (int)(i / per_tile);
    const int e = (int)(i - (long)t * per_tile) * 8;
    const int r = e / BN, c = e - r * BN;
    int tm, tn;
    wg_tile(tile0 + t, M / BM, N / BN, map, group_m, tm, tn);
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < S; ++sp) {
      const float* p = part + ((long)sp * ntile + t) * BM * BN + e;
      const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
    OT* o = C + ((long)tm * BM + r) * ldc + (long)tn * BN + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = from_f<OT>(accumulate ? to_f(o[j]) + v[j] : v[j]);
  }
}

// tile map and group depth: the shipped defaults, changed only through set_gemm_tile_maps (the
// placement A/B of profiles/r5/kernel_experiments.md and the map tests)
static int g_wg_map = 0, g_wg_gm = GROUP_M;
static void wg_knobs(int& map, int& gm) {
  map = g_wg_map;
  gm = g_wg_gm;
}

template <typename T, typename OT>
void launch4(const void* a, long lda, const void* b, long ldb, void* c, long ldc, long c_split, int M, int N, int K,
             int S, bool accumulate, hipStream_t s, int tile0 = 0, int ntile = -1, int compact = 0) {
  static const bool attr = hipFuncSetAttribute((const void*)wgrad4_k<T, OT>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
  (void)attr;
  const int cnt = ntile < 0 ? (M / BM) * (N / BN) : ntile;
  const dim3 grid(cnt, S);
  const bool wide = reinterpret_cast<uintptr_t>(c) % 16 == 0 && (ldc * (long)sizeof(OT)) % 16 == 0 &&
                    (c_split * (long)sizeof(OT)) % 16 == 0;
  int map, gm;
  wg_knobs(map, gm);
  hipLaunchKernelGGL((wgrad4_k<T, OT>), grid, dim3(g4::THREADS4), LDS_BYTES, s, (const T*)a, lda, (const T*)b, ldb,
                     (OT*)c, ldc, c_split, M, N, K, (int)accumulate, (int)wide, map, gm, tile0, ntile, compact);
}

template <typename T, typename OT, bool AK = false>
void launch_v(const void* a, long lda, const void* b, long ldb, void* c, long ldc, long c_split, int M, int N, int K,
              int S, bool accumulate, hipStream_t s) {
  static const bool attr = hipFuncSetAttribute((const void*)wgrad_gemm_k<T, OT, AK>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
  (void)attr;
  const dim3 grid((M / BM) * (N / BN), S);
  const bool wide = reinterpret_cast<uintptr_t>(c) % 16 == 0 && (ldc * (long)sizeof(OT)) % 16 == 0 &&
                    (c_split * (long)sizeof(OT)) % 16 == 0;
  hipLaunchKernelGGL((wgrad_gemm_k<T, OT, AK>), grid, dim3(Geo::THREADS), LDS_BYTES, s, (const T*)a, lda,
                     (const T*)b, ldb, (OT*)c, ldc, c_split, M, N, K, (int)accumulate, (int)wide);
}

// wgrad4_k (1.02-1.06x wgrad_gemm_k on the Llama-3-8B / Llama-3.2-1B / GPT2-774M weight
// gradients at 40,960 tokens, profiles/r3/wgrad4_vs_v2.jsonl) except for deep split-K (S >= 8:
// GPT2-774M's 1280 x 1280 o-projection, 200 workgroups), where wgrad_gemm_k was 12 % faster
template <typename T, typename OT>
void launch(const void* a, long lda, const void* b, long ldb, void* c, long ldc, long c_split, int M, int N, int K,
            int S, bool accumulate, hipStream_t s) {
  if (S >= 8) launch_v<T, OT>(a, lda, b, ldb, c, ldc, c_split, M, N, K, S, accumulate, s);
  else launch4<T, OT>(a, lda, b, ldb, c, ldc, c_split, M, N, K, S, accumulate, s);
}

}  // namespace

void set_wgrad_tile_map(int map, int group_m) {
  g_wg_map = map;
  g_wg_gm = group_m > 0 ? group_m : GROUP_M;
}

bool gemm_nn_supported(int M, int N, int K) { return M > 0 && N > 0 && M % BM == 0 && N % BN == 0 && K >= KCH && K % KCH == 0; }

void gemm_nn(DType dt, DType odt, const void* a, long lda, const void* b, long ldb, void* c, long ldc, int M, int N,
             int K, bool accumulate, hipStream_t s) {
  BLLM_DISPATCH(odt, OT, {
    if (dt == DType::BF16) launch_v<bf16_t, OT, true>(a, lda, b, ldb, c, ldc, 0, M, N, K, 1, accumulate, s);
    else launch_v<f16_t, OT, true>(a, lda, b, ldb, c, ldc, 0, M, N, K, 1, accumulate, s);
  });
}

bool wgrad_gemm_supported(int M, int N, int K, int S) {
  return M > 0 && N > 0 && M % BM == 0 && N % BN == 0 && K >= KCH && K % KCH == 0 && S >= 1 && S <= K / KCH;
}

bool wgrad_tail_supported(int M, int N, int K, int full, int St) {
  const int tiles = M > 0 && N > 0 && M % BM == 0 && N % BN == 0 ? (M / BM) * (N / BN) : 0;
  return tiles > 0 && full >= 0 && full < tiles && K >= KCH && K % KCH == 0 && St >= 2 && St <= K / KCH;
}

// dW with the grouped tile order split in two launches: tiles [0, full) whole-K straight into c
// (full = whole waves of workgroups), the tail [full, tiles) split St ways over K into compact
// fp32 partials (part: St * (tiles - full) * 256 * 256 floats), summed into c by wg_tail_sum_k.
// Same wave count as splitting every tile, ~1/St of its partial traffic when the tail is short.
void wgrad_gemm_tail(DType dt, DType odt, const void* a, long lda, const void* b, long ldb, void* c, long ldc, int M,
                     int N, int K, int full, int St, float* part, bool accumulate, hipStream_t s) {
  const int tail = (M / BM) * (N / BN) - full;
  int map, gm;
  wg_knobs(map, gm);
  BLLM_DISPATCH(odt, OT, {
    if (full > 0) {
      if (dt == DType::BF16) launch4<bf16_t, OT>(a, lda, b, ldb, c, ldc, 0, M, N, K, 1, accumulate, s, 0, full, 0);
      else launch4<f16_t, OT>(a, lda, b, ldb, c, ldc, 0, M, N, K, 1, accumulate, s, 0, full, 0);
    }
    if (dt == DType::BF16) launch4<bf16_t, float>(a, lda, b, ldb, part, BN, 0, M, N, K, St, false, s, full, tail, 1);
    else launch4<f16_t, float>(a, lda, b, ldb, part, BN, 0, M, N, K, St, false, s, full, tail, 1);
    const long work = (long)tail * BM * BN / 8;
    const int g = (int)((work + 255) / 256 < 2048 ? (work + 255) / 256 : 2048);
    hipLaunchKernelGGL((wg_tail_sum_k<OT>), dim3(g), dim3(256), 0, s, (const float*)part, (OT*)c, ldc, M, N, full, tail,
                       St, map, gm, (int)accumulate);
  });
}

void wgrad_gemm(DType dt, DType odt, const void* a, long lda, const void* b, long ldb, void* c, long ldc,
                long c_split, int M, int N, int K, int S, bool accumulate, hipStream_t s) {
  BLLM_DISPATCH(odt, OT, {
    if (dt == DType::BF16) launch<bf16_t, OT>(a, lda, b, ldb, c, ldc, c_split, M, N, K, S, accumulate, s);
    else launch<f16_t, OT>(a, lda, b, ldb, c, ldc, c_split, M, N, K, S, accumulate, s);
  });
}

}  // namespace bllm
