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
//  * tile 256 x 256 per workgroup (8 waves = 2 (M) x 4 (N), 128 x 64 outputs per wave,
//    acc[8][4] of 16x16 fp32 fragments), one 32-deep k-step per LDS ring slot;
//  * a ring of 4 slots (A [32 k][256 m] + B [32 k][256 n] images, 16 KiB each, 128 KiB total)
//    filled by LDS-DMA (global_load_lds_dwordx4, 4 per lane per slot) 3 slots ahead of the
//    MFMAs; one raw s_barrier per slot, counted vmcnt (never drained to 0 inside the loop);
//  * fragments are read with ds_read_b64_tr_b16 (a 16-lane group gets 4 k-rows x 16 columns
//    delivered column-major = 4 k-values of one m/n column per lane); two reads give the 8
//    k-values of a 16x16x32 A or B fragment;
//  * bank conflicts: a 32-lane half-wave reads 8 k-rows x 32 B at the same columns; the image
//    XOR-permutes 16-B chunks within each 512-B k-row by f(r) = 2*((r&3) | ((r>>3)&1)<<2), which
//    puts the 8 rows on 8 distinct 32-B bank groups (conflict-free).  The DMA writes LDS
//    lane-linearly, so the permutation is applied to the per-lane GLOBAL source address (a
//    permutation of 16-B chunks inside one 512-B row: the loads stay fully coalesced);
//  * blockIdx.x -> tile: XCD-aware (each XCD gets a contiguous range of tiles, bijective for
//    any count), grouped 8 tile-rows deep so the 32 tiles an XCD runs at once share 8 A and 4 B
//    panels in its L2;
//  * blockIdx.y = split-K index (few-tile GEMMs): split s reduces its own 128-aligned token
//    range into fp32 partial s of C (c_split elements apart), summed afterwards in a fixed
//    order — deterministic either way (each output element has one owner per split).
#include <stdlib.h>

#include <type_traits>

#include "api.h"

namespace bllm {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  static __device__ __forceinline__ f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
};
template <> struct Mfma<f16_t> {
  static __device__ __forceinline__ f32x4 run(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
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
constexpr int THREADS = 512;
constexpr int GROUP_M = 8;

__device__ __forceinline__ int swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

__device__ __forceinline__ s16x8 frag(const char* p) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * ROWB));
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <typename T, typename OT, int VAR>
__global__ __launch_bounds__(THREADS) void wgrad_gemm_k(const T* __restrict__ A, long lda, const T* __restrict__ B,
                                                        long ldb, OT* __restrict__ C, long ldc, long c_split, int M,
                                                        int N, int K, int accumulate) {
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

  // ---- staging: lane-linear LDS rows, XOR-permuted global chunks (loop-invariant offsets)
  uint32_t voffA[2], voffB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = (wave * 2 + j) * 2 + (lane >> 5), c = (lane & 31) ^ swz(r);
    voffA[j] = (uint32_t)((r * lda + 8 * c) * (long)sizeof(T));
    voffB[j] = (uint32_t)((r * ldb + 8 * c) * (long)sizeof(T));
  }
  const uint32_t lds0 = lds_u32(smem);
  const T* Abase = A + (long)c_lo * KCH * lda + m0;
  const T* Bbase = B + (long)c_lo * KCH * ldb + n0;
  auto stage = [&](int kt, int slot) {
    const void* a = sgpr_ptr(Abase + (long)kt * BK * lda);
    const void* b = sgpr_ptr(Bbase + (long)kt * BK * ldb);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      glds16s(a, voffA[j], lds0 + slot * SLOTB + (wave * 2 + j) * 1024);
      glds16s(b, voffB[j], lds0 + B_BASE + slot * SLOTB + (wave * 2 + j) * 1024);
    }
  };

  // ---- fragment read offsets: lane (g, q, p) reads k-row 8g + q (+4), columns 4p..4p+3
  const int g = lane >> 4, qq = (lane & 15) >> 2, p = lane & 3;
  const int f = 2 * (qq | ((g & 1) << 2));  // == swz(8g + qq + 4h) for h = 0, 1
  const int wm = wave >> 2, wn = wave & 3;
  const int rowb = (8 * g + qq) * ROWB + (p & 1) * 8 + (p >> 1) * 16;
  int aoff[8], boff[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) aoff[i] = rowb + (wm * 16 + ((2 * i) ^ f)) * 16;
#pragma unroll
  for (int j = 0; j < 4; ++j) boff[j] = B_BASE + rowb + ((wn * 8 + 2 * j) ^ f) * 16;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (VAR == 1) {
    // Fragments of slot kt+1 are read into the second register set WHILE slot kt's MFMAs
    // run, so no wave waits on LDS latency after a barrier: the MFMA pipe stays fed across it.
    // Ring: DMA of k-slot kt+4 refills LDS slot kt as soon as every wave holds slot kt in VGPRs.
    struct Frags { s16x8 a[8], b[4]; };
    auto load = [&](Frags& F, int slot) {
      const char* base = smem + slot * SLOTB;
#pragma unroll
      for (int j = 0; j < 4; ++j) F.b[j] = frag(base + boff[j]);
#pragma unroll
      for (int i = 0; i < 8; ++i) F.a[i] = frag(base + aoff[i]);
    };
    // G.b first, then G.a[i] just before F.a[i]'s MFMAs: F.a[i] dies as G.a[i] arrives, so the
    // two sets cost 8 B-fragments + 9 A-fragments of VGPRs, not 2 x 12.  The loop body is
    // branch-free (the final trip is peeled) so hipcc's lgkmcnt counting stays exact.
    auto it = [&](auto wait_n, auto do_stage, auto last, int kt, Frags& F, Frags& G) {
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
        for (int j = 0; j < 4; ++j) G.b[j] = frag(nxt + boff[j]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (!LAST) G.a[i] = frag(nxt + aoff[i]);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = Mfma<T>::run(F.a[i], F.b[j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    };
    using W8 = std::integral_constant<int, 8>;
    using W4 = std::integral_constant<int, 4>;
    using W0 = std::integral_constant<int, 0>;
    using Y = std::true_type;
    using Nn = std::false_type;
    stage(0, 0);
    stage(1, 1);
    stage(2, 2);
    stage(3, 3);
    vm_wait<12>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    Frags F0, F1;
    load(F0, 0);
    int kt = 0;
    for (; kt < nk - NSLOT; kt += NSLOT) {
      it(W8{}, Y{}, Nn{}, kt + 0, F0, F1);
      it(W8{}, Y{}, Nn{}, kt + 1, F1, F0);
      it(W8{}, Y{}, Nn{}, kt + 2, F0, F1);
      it(W8{}, Y{}, Nn{}, kt + 3, F1, F0);
    }
    it(W8{}, Nn{}, Nn{}, kt + 0, F0, F1);
    it(W4{}, Nn{}, Nn{}, kt + 1, F1, F0);
    it(W0{}, Nn{}, Nn{}, kt + 2, F0, F1);
    it(W0{}, Nn{}, Y{}, kt + 3, F1, F0);
  } else {
  stage(0, 0);
  stage(1, 1);
  stage(2, 2);

  auto step = [&](int kt, int slot) {
    const int rem = nk - 1 - kt;  // slots still in flight behind this one
    if (rem >= 2) vm_wait<8>();
    else if (rem == 1) vm_wait<4>();
    else vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot kt-1 are done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // no LDS read of slot kt is hoisted above the barrier
    if (kt + 3 < nk) stage(kt + 3, (slot + 3) & (NSLOT - 1));
    const char* base = smem + slot * SLOTB;
    s16x8 bf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = frag(base + boff[j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const s16x8 af = frag(base + aoff[i]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = Mfma<T>::run(af, bf[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  for (int kt = 0; kt < nk; kt += NSLOT) {
    step(kt + 0, 0);
    step(kt + 1, 1);
    step(kt + 2, 2);
    step(kt + 3, 3);
  }
  }

  // ---- epilogue: lane holds C[16i + 4(l>>4) + e][16j + (l&15)] of the wave's 128 x 64 block
  OT* c = C + sp * c_split + (m0 + wm * 128 + 4 * (lane >> 4)) * ldc + n0 + wn * 64 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        OT* o = c + (long)(16 * i + e) * ldc + 16 * j;
        const float v = acc[i][j][e];
        *o = from_f<OT>(accumulate ? to_f(*o) + v : v);
      }
}

template <typename T, typename OT, int VAR>
void launch_v(const void* a, long lda, const void* b, long ldb, void* c, long ldc, long c_split, int M, int N, int K,
              int S, bool accumulate, hipStream_t s) {
  static const bool attr = hipFuncSetAttribute((const void*)wgrad_gemm_k<T, OT, VAR>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
  (void)attr;
  const dim3 grid((M / BM) * (N / BN), S);
  hipLaunchKernelGGL((wgrad_gemm_k<T, OT, VAR>), grid, dim3(THREADS), LDS_BYTES, s, (const T*)a, lda, (const T*)b,
                     ldb, (OT*)c, ldc, c_split, M, N, K, (int)accumulate);
}

// BLLM_WGRAD_VARIANT: 0 = fragments read after each barrier, 1 = next slot's fragments read
// under the current slot's MFMAs (two register sets)
int variant() {
  static const int v = [] {
    const char* e = getenv("BLLM_WGRAD_VARIANT");
    return e ? atoi(e) : 1;
  }();
  return v;
}

template <typename T, typename OT>
void launch(const void* a, long lda, const void* b, long ldb, void* c, long ldc, long c_split, int M, int N, int K,
            int S, bool accumulate, hipStream_t s) {
  if (variant() == 0) launch_v<T, OT, 0>(a, lda, b, ldb, c, ldc, c_split, M, N, K, S, accumulate, s);
  else launch_v<T, OT, 1>(a, lda, b, ldb, c, ldc, c_split, M, N, K, S, accumulate, s);
}

}  // namespace

bool wgrad_gemm_supported(int M, int N, int K, int S) {
  return M > 0 && N > 0 && M % BM == 0 && N % BN == 0 && K >= KCH && K % KCH == 0 && S >= 1 && S <= K / KCH;
}

void wgrad_gemm(DType dt, DType odt, const void* a, long lda, const void* b, long ldb, void* c, long ldc,
                long c_split, int M, int N, int K, int S, bool accumulate, hipStream_t s) {
  BLLM_DISPATCH(odt, OT, {
    if (dt == DType::BF16) launch<bf16_t, OT>(a, lda, b, ldb, c, ldc, c_split, M, N, K, S, accumulate, s);
    else launch<f16_t, OT>(a, lda, b, ldb, c, ldc, c_split, M, N, K, S, accumulate, s);
  });
}

}  // namespace bllm
