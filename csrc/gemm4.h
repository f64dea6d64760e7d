// Shared pieces of the 4-wave (one wave per SIMD, 128 x 128 outputs per wave) MFMA GEMMs:
// csrc/gemm_nt.hip (forward layout) and csrc/gemm_wgrad.hip (weight-gradient layout).
#pragma once
#include "common.h"

namespace bllm {
namespace g4 {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int TN = 256;          // output tile columns (and rows)
constexpr int THREADS4 = 256;    // 4 waves
enum { EPI_NONE = 0, EPI_SWIGLU = 1, EPI_ROPE = 2, EPI_BIAS_GELU = 3 };

// MFMA with the accumulator tied in place in an AGPR ("+a"): hipcc otherwise renames the
// 256 accumulators of the 4-wave kernel between unrolled steps and pays for it in
// v_accvgpr_read/write copies.  Operand hazards: fragments come from ds_read (waited for by the
// compiler's lgkmcnt, no VALU producer); a chain on one accumulator needs no padding; the first
// compiler reader after the last MFMA is behind mfma_drain().
template <typename T> struct MfA;
template <> struct MfA<bf16_t> {
  static __device__ __forceinline__ void run(f32x4& c, const s16x8& a, const s16x8& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  }
  // c = 0 in place (srcC the inline constant 0, A = B = 0): resets an accumulator without
  // letting hipcc re-home it
  static __device__ __forceinline__ void zero(f32x4& c, const s16x8& z) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "+a"(c) : "v"(z));
  }
};
template <> struct MfA<f16_t> {
  static __device__ __forceinline__ void run(f32x4& c, const s16x8& a, const s16x8& b) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  }
  static __device__ __forceinline__ void zero(f32x4& c, const s16x8& z) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %1, 0" : "+a"(c) : "v"(z));
  }
};
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

// One LDS-DMA piece: buffer_load_dwordx4 ... offen lds on a loop-invariant descriptor of the
// wave's rows, the tile advance in soffset, m0 written without save / restore (nothing else in the
// kernel uses m0).  The alternatives measured in round 3 (global_load_lds with saddr, sc0 sc1 and nt
// cache policies) were no faster and were removed.
template <int DV>
__device__ __forceinline__ void bdma16(const i32x4& rsrc, uint32_t voff, uint32_t soff, uint32_t lds_dst) {
  static_assert(DV == 1, "only the offen descriptor form is kept");
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
               ::"v"(voff), "s"(rsrc), "s"(soff), "s"(lds_dst) : "memory");
}
// raw buffer descriptor (stride 0, no bounds limit) of a wave-uniform base pointer
__device__ __forceinline__ i32x4 make_rsrc(const void* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  return i32x4{(int)__builtin_amdgcn_readfirstlane((uint32_t)v),
               (int)(__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) & 0xFFFF), (int)0xFFFFFFFF, 0x00020000};
}

// Operands are swapped in the MFMAs (src A = the B fragment), so lane l of acc[I][J] holds the
// 4 CONSECUTIVE columns 16J + 4(l>>4) .. +3 of row 16I + (l&15) of its wave's 128 x 128 block.
// Epilogue, 16-bit output, no accumulate, no SwiGLU: the whole 256 x 256 tile is staged in LDS as
// bf16/fp16 in one pass (one ds_write_b64 per accumulator; 16-B chunk c of row r at c ^ (r & 15),
// conflict-free for the writes' 16-row lane groups) and leaves as 16-B row-contiguous stores.
// Otherwise fp32 staging in two 128-row passes (ds_write_b128 per accumulator, chunk ^ (r & 7)).
template <typename T, typename OT, int EPI>
__device__ __forceinline__ void epilogue4(f32x4 (&acc)[8][8], char* smem, int wm, int wn, int lane, OT* C, long ldc,
                                          long m0, long n0, long g0, long u0, int accumulate, int wide, OT* act,
                                          int F) {
  OT* cbase = C + m0 * ldc + n0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if constexpr (sizeof(OT) == 2 && EPI == EPI_NONE) {
    if (wide && !accumulate) {
      constexpr int RB = TN * 2;   // 512 B: 32 chunks of 8 elements
      typedef short s16x4v __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int I = 0; I < 8; ++I)
#pragma unroll
        for (int J = 0; J < 8; ++J) {
          const int r = 128 * wm + 16 * I + (lane & 15);
          const int col = 128 * wn + 16 * J + 4 * (lane >> 4);          // 4 columns, half a chunk
          const int ch = (col >> 3) ^ (r & 15);
          s16x4v w;
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = __builtin_bit_cast(short, from_f<OT>(acc[I][J][e]));
          *(s16x4v*)(smem + r * RB + ch * 16 + (col & 4) * 2) = w;
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll 8
      for (int tr = 0; tr < 256 * 32 / THREADS4; ++tr) {
        const int q = (int)threadIdx.x + tr * THREADS4;
        const int r = q >> 5, c = q & 31;
        const uint4 v = *(const uint4*)(smem + r * RB + ((c ^ (r & 15)) << 4));
        *(uint4*)(cbase + (long)r * ldc + 8 * c) = v;
      }
      return;
    }
  }
  if (wide) {
    constexpr int RB = TN * 4;
    constexpr int EPT = 16 / (int)sizeof(OT);
    constexpr int NCH = EPT / 4;
    constexpr int IPR = TN / EPT;
    constexpr int TRIPS = 128 * IPR / THREADS4;
    struct alignas(16) V16 { OT e[EPT]; };
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (wm == pass) {
#pragma unroll
        for (int I = 0; I < 8; ++I)
#pragma unroll
          for (int J = 0; J < 8; ++J) {
            const int lr = 16 * I + (lane & 15), col = wn * 128 + 16 * J + 4 * (lane >> 4);
            *(f32x4*)(smem + lr * RB + (((col >> 2) ^ (lr & 7)) << 4)) = acc[I][J];
          }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll 4
      for (int tr = 0; tr < TRIPS; ++tr) {
        const int q = (int)threadIdx.x + tr * THREADS4;
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
        constexpr int AIPR = 128 / EPT;
        constexpr int ATRIPS = 128 * AIPR / THREADS4;
#pragma unroll 4
        for (int tr = 0; tr < ATRIPS; ++tr) {
          const int q = (int)threadIdx.x + tr * THREADS4;
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
            w.e[k] = from_f<OT>(a * silu_sig(a) * b);
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
  OT* c = cbase + (128 * wm + (lane & 15)) * ldc + 128 * wn + 4 * (lane >> 4);
#pragma unroll
  for (int I = 0; I < 8; ++I)
#pragma unroll
    for (int J = 0; J < 8; ++J)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        OT* o = c + (long)(16 * I) * ldc + 16 * J + e;
        *o = from_f<OT>((accumulate ? to_f(*o) : 0.f) + acc[I][J][e]);
      }
}

}  // namespace g4
}  // namespace bllm
