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
// delta = rowsum(dO * O) is computed by the dQ kernel (which holds dO in registers anyway
// and runs first) and handed to the dK/dV kernel through a [B,H,T] fp32 buffer.  Q/dO (dK/dV
// kernel) and K/V (dQ kernel) tiles arrive by global_load_lds DMA, double-buffered, stored as
// 16-B-chunk XOR images for MFMA row reads and 64-B-chunk XOR images for hardware-transposed
// reads (ds_read_b64_tr_b16).  Causal: only tiles at/below the diagonal; heaviest first.
#include <float.h>
#include <stdlib.h>
#include <type_traits>

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
// ONE image of a [rows][HD] tile serving both 16-B row reads (ds_read_b128, S / dP operands)
// and hardware-transposed reads (ds_read_b64_tr_b16, dV^T / dK^T operands): chunk ch of row r at
// ch ^ f(r).  HD 128 (256-B rows): f = ((r&3)<<2) | ((r>>2)&3)  (cdna_hip_programming.md T10 (b)).
// HD 64 (128-B rows): f = (((r>>1)&1)<<2) | ((r>>2)&3) -- over the 8 same-parity rows of every
// b128 lane group f is a permutation of 0..7 (row reads conflict-free), and rows r, r+2 of an
// aligned 4-row block differ in bit 2 (the 4-chunk block a transposed half-wave read touches),
// so a 32-lane transposed read hits 32 distinct bank pairs.  Depends on r & 15 only.
template <int HD> __device__ __forceinline__ int dual_f(int r) {
  if constexpr (HD == 128) return ((r & 3) << 2) | ((r >> 2) & 3);
  else return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
}
template <int HD> __device__ __forceinline__ int dual_off(int r, int ch) {
  return r * (HD * 2) + ((ch ^ dual_f<HD>(r)) << 4);
}

// dS image [32 q][128 keys] bf16: 16-B chunk XOR by q
__device__ __forceinline__ int ds_off(int q, int key) {
  return q * 256 + ((((key >> 3) ^ (q & 15))) << 4) + ((key & 7) << 1);
}

// two floats -> packed pair (one v_cvt_pk_bf16_f32 for bf16)
template <typename T> __device__ __forceinline__ uint32_t pk2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef T t2 __attribute__((ext_vector_type(2)));
  const t2 v = __builtin_convertvector((f2{a, b}), t2);
  uint32_t u;
  __builtin_memcpy(&u, &v, 4);
  return u;
}

template <typename v8> __device__ __forceinline__ v8 tr8(const char* base, int off_lo, int off_hi) {
  const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off_lo));
  const s16x4 r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off_hi));
  // whole-register concatenation (an element-wise short[8] build made hipcc emit a v_bfi per
  // fragment and wait for the read right there)
  return __builtin_bit_cast(v8, __builtin_shufflevector(r1, r2, 0, 1, 2, 3, 4, 5, 6, 7));
}
}  // namespace

constexpr int BWD_BKV = 128;  // keys per workgroup
constexpr int BWD_BQ = 32;    // queries per step
constexpr float kLog2eB = 1.4426950408889634f;

// LDS bytes of one ring slot of the dK/dV kernel: Q rows, Q^T image, dO rows, dO^T image,
// and a per-wave copy of the step's lse/delta (so each wave's stats DMA is its own)
template <int HD, bool DUAL = false, bool MASK = false> constexpr int dkdv_buf_bytes() {
  return (DUAL ? 2 : 4) * BWD_BQ * HD * 2 + 4 * 256 + (MASK ? 4 * 256 : 0);
}

// Instruction budget per 32-query step (per wave): 32 MFMAs, 16 b128 + 32 tr_b64 LDS reads at
// loop-invariant per-lane offsets (+ a per-slot base), ~60 VALU of softmax math (the 1/sqrt(d)
// of dS is folded into the final dK), 9 saddr LDS-DMA issues whose per-lane offsets are
// precomputed.  Masking (causal diagonal, sequence tail) and dropout are compile-time variants
// so the common interior step carries no per-element branches.
// FUSEG: one workgroup sweeps all H/G query heads of its kv head (dK/dV summed in registers,
// written once in bf16: no fp32 per-head partials, no reduction kernel); otherwise one query
// head per workgroup plus the attn_bwd_kv_reduce_k pass for GQA.
// DUAL: Q and dO each staged as ONE dual-use image (dual_off) instead of a row image plus a
// transposed image: half the LDS and DMA per step, which buys a 4-slot ring (three steps in
// flight) at two workgroups per CU -- the 2-slot version waits on its DMA ~60 % of wave cycles.
// MASK (with DROP): the dropout keep bits come from the forward's keep mask -- one more 4-byte
// DMA per wave and step brings the 32 words (queries of the step, this wave's 32 keys) into the
// slot -- instead of one counter hash per (query, key) element.
// VLDS: the V fragments (B operands of dP = dO V^T) live in LDS -- [32 keys][HD] per wave,
// 16-B chunks XOR-swizzled by row (r_off) -- instead of 32 VGPRs for the whole kernel: at hd 128
// K + V fragments (64) + dK/dV accumulators (128) + S/dP (32) leave too little of the 256 VGPRs
// two waves per SIMD allow, and hipcc spilled the fragments to scratch, reloading them every
// step behind an s_waitcnt vmcnt(0) that also drained the Q/dO DMA ring.
// Inverse RoPE in a backward epilogue (rotate_half form, reference common_components.py:6-35):
// the lane holds elements d..d+3 (d = dc + 8 gq + 4 hh) of the first half in lo and the same
// elements of the second half (d + HD/2) in hi, so each rotation pair is lane-local:
//   g1' = g1 c + g2 s,  g2' = g2 c - g1 s   (c, s = cos/sin [T, HD/2] fp32 at position pos).
// Replaces a separate rope pass over dQ / dK (read + write of [N, (H + G) hd]).  ``row`` is the
// head's first element.
// One row-per-lane-pair 16-B store (cdna_hip_programming.md T21): this lane holds the packed
// columns of groups gq (a) and gq+1 (b), 4 each, 4 hh + 0..3 within the group; one
// v_permlane32_swap per dword leaves group gq's 8 columns in the lower lane half and gq+1's in the
// upper, stored at dst = row + 8 gq + 8 hh.  Lanes l and l+32 must hold the same row.
template <typename T>
__device__ __forceinline__ void store16_pair(T* dst, const uint32_t (&a)[2], const uint32_t (&b)[2]) {
  const auto rx = __builtin_amdgcn_permlane32_swap(a[0], b[0], false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(a[1], b[1], false, false);
  *reinterpret_cast<uint4*>(dst) = uint4{rx[0], ry[0], rx[1], ry[1]};
}

template <typename T, int HD>
__device__ __forceinline__ void rope_bwd_store(const f32x16& lo, const f32x16& hi, float scale, int hh, int pos,
                                               int dc, const float* __restrict__ rcos,
                                               const float* __restrict__ rsin, T* row) {
  constexpr int HALF = HD / 2;
  const float* cp = rcos + (long)pos * HALF + dc + 4 * hh;
  const float* sp = rsin + (long)pos * HALF + dc + 4 * hh;
  uint32_t w1[4][2], w2[4][2];  // packed (d, d+1), (d+2, d+3) of group gq, both halves
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    const float4 c = *reinterpret_cast<const float4*>(cp + 8 * gq);
    const float4 sn = *reinterpret_cast<const float4*>(sp + 8 * gq);
    const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
    float o1[4], o2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float g1 = lo[4 * gq + j] * scale, g2 = hi[4 * gq + j] * scale;
      o1[j] = g1 * cc[j] + g2 * ss[j];
      o2[j] = g2 * cc[j] - g1 * ss[j];
    }
    w1[gq][0] = pk2<T>(o1[0], o1[1]);
    w1[gq][1] = pk2<T>(o1[2], o1[3]);
    w2[gq][0] = pk2<T>(o2[0], o2[1]);
    w2[gq][1] = pk2<T>(o2[2], o2[3]);
  }
  // 16-B stores (T21, as attn_fwd_mfma_k's epilogue): lanes l and l+32 hold the same row
#pragma unroll
  for (int gq = 0; gq < 4; gq += 2) {
    store16_pair<T>(row + dc + 8 * gq + 8 * hh, w1[gq], w1[gq + 1]);
    store16_pair<T>(row + HALF + dc + 8 * gq + 8 * hh, w2[gq], w2[gq + 1]);
  }
}

template <typename T, int HD, bool DROP, int NBUF, int OCC, bool FUSEG = false, bool DUAL = false, bool MASK = false,
          bool VLDS = false>
__global__ __launch_bounds__(256, OCC) void attn_bwd_mfma_k(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ delta, T* __restrict__ dqkv,
                                                            float* __restrict__ dkv_part, int T_, int H, int G, int B_,
                                                            bool causal, uint32_t thr, float inv_keep,
                                                            uint64_t seed, uint64_t doff,
                                                            const uint32_t* __restrict__ kmask,
                                                            const float* __restrict__ rcos,
                                                            const float* __restrict__ rsin, int xmap) {
  typedef typename MFb<T>::v8 v8;
  constexpr int KK = HD / 16, DT = HD / 32, CH = HD / 8, ROWB = HD * 2;
  constexpr int IMG = BWD_BQ * ROWB;            // bytes of one [32][HD] image
  constexpr int PPW = IMG / 1024 / 4;           // 1-KiB DMA pieces per wave per image
  constexpr int PROWS = 256 / CH;               // rows between a wave's consecutive pieces
  static_assert(!MASK || DROP, "keep mask only with dropout");
  constexpr int BUF = dkdv_buf_bytes<HD, DUAL, MASK>();
  constexpr int NIMG = DUAL ? 2 : 4;            // LDS images per step
  constexpr int NPW = NIMG * PPW + 1 + (MASK ? 1 : 0);  // DMA instructions per wave per step
  static_assert(NBUF >= 2 && NBUF <= 4, "ring depth");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // heaviest (lowest) key block first across the whole grid; all key blocks of one (b, h)
  // share lin % 8, i.e. one XCD and its L2 (Q / dO re-reads hit there)
  const int lin = blockIdx.x, nbh = (FUSEG ? G : H) * B_;
  int kb, bh;
  attn_wg_order(lin, nbh, 1, xmap, kb, bh);
  const int rep = H / G;
  const int b = FUSEG ? bh / G : bh / H;
  const int g = FUSEG ? bh % G : (bh % H) / rep;
  const int h_first = FUSEG ? g * rep : bh % H, h_count = FUSEG ? rep : 1;
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar branches)
  const long rs = (long)(H + 2 * G) * HD;
  const long ors = (long)H * HD;
  const T* kb_ = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const T* vb_ = qkv + (long)b * T_ * rs + (long)(H + G + g) * HD;
  const int k0 = kb * BWD_BKV;
  const int kw0 = k0 + 32 * w;
  const int mykey = kw0 + l32;
  const float scale = rsqrtf((float)HD), c = scale * kLog2eB;

  // ---- K / V fragments of this wave's 32 keys (B operands, key = lane column)
  constexpr int VOFF = NBUF * BUF;              // VLDS: per-wave V rows after the ring
  v8 kf[KK], vf[VLDS ? 1 : KK];
  {
    const int kr = mykey < T_ ? mykey : T_ - 1;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      kf[kk] = *reinterpret_cast<const v8*>(kb_ + (long)kr * rs + kk * 16 + hh * 8);
      const v8 vv = *reinterpret_cast<const v8*>(vb_ + (long)kr * rs + kk * 16 + hh * 8);
      if constexpr (VLDS)
        *reinterpret_cast<v8*>(smem + VOFF + w * 32 * ROWB + r_off<HD>(l32, kk * 2 + hh)) = vv;
      else
        vf[kk] = vv;
    }
    // consume the fragments here: the compiler then retires these loads before the loop and
    // inserts no vmcnt waits inside it (it cannot see the asm-issued DMA, whose counts the
    // loop manages itself)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) asm volatile("" ::"v"(kf[kk]));
    if constexpr (!VLDS) {
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) asm volatile("" ::"v"(vf[kk]));
    }
  }
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) { dk[i] = f32x16{}; dv[i] = f32x16{}; }

  // DMA source offsets of this lane's piece (j = 0; piece j adds j*PROWS rows, folded into the
  // uniform SGPR base), one for the row image and one for the transposed image
  uint32_t q_r, q_t, o_r, o_t;
  {
    const int P = w * 64 + lane;
    const int r = P / CH, pc = P % CH;
    int rc;
    if constexpr (DUAL) rc = pc ^ dual_f<HD>(r);
    else if constexpr (HD == 128) rc = pc ^ (r & 15);
    else rc = pc ^ ((r >> 1) & 7);
    const int c64 = (pc >> 2) ^ (HD == 128 ? (r & 3) : ((r >> 1) & 1));
    const int tc = c64 * 4 + (pc & 3);
    q_r = (uint32_t)(r * rs * 2 + rc * 16);
    q_t = (uint32_t)(r * rs * 2 + tc * 16);
    o_r = (uint32_t)(r * ors * 2 + rc * 16);
    o_t = (uint32_t)(r * ors * 2 + tc * 16);
  }
  // image offsets inside a slot: Q rows, Q^T, dO rows, dO^T (DUAL: Q at 0, dO at IMG)
  constexpr int IQT = DUAL ? 0 : IMG, IOR = DUAL ? IMG : 2 * IMG, IOT = DUAL ? IMG : 3 * IMG;
  constexpr int ISTAT = NIMG * IMG;
  constexpr int IMASK = ISTAT + 4 * 256;         // per-wave keep-mask words (MASK)
  const long kw_row = (long)((T_ + 31) / 32) * T_;  // keep-mask words per (b, h)
  const uint32_t smem_u = lds_u32(smem);
  for (int hi = 0; hi < h_count; ++hi) {
  const int h = h_first + hi;
  const T* qb_ = qkv + (long)b * T_ * rs + (long)h * HD;
  const T* ob_ = dout + (long)b * T_ * ors + (long)h * HD;
  const float* lse_ = lse + ((long)b * H + h) * T_;
  const float* del_ = delta + ((long)b * H + h) * T_;
  const float* stat_src = (lane < 32 ? lse_ : del_);
  DropSlab ds;
  uint64_t dslab = 0;
  if constexpr (DROP) {
    dslab = doff + (uint64_t)(b * H + h) * T_ * T_;
    ds.init(seed, dslab);
  }

  // DMA of one 32-query step into ring slot `slot`
  auto issue = [&](int q0, int slot) {
    const uint32_t base = smem_u + slot * BUF;
    if (q0 + BWD_BQ <= T_) {
#pragma unroll
      for (int j = 0; j < PPW; ++j) {
        const void* qs = sgpr_ptr(qb_ + (long)(q0 + j * PROWS) * rs);
        const void* os = sgpr_ptr(ob_ + (long)(q0 + j * PROWS) * ors);
        const uint32_t pd = (w + 4 * j) * 1024;
        glds16s(qs, q_r, base + pd);
        if constexpr (!DUAL) glds16s(qs, q_t, base + IQT + pd);
        glds16s(os, o_r, base + IOR + pd);
        if constexpr (!DUAL) glds16s(os, o_t, base + IOT + pd);
      }
    } else {  // sequence tail: clamp rows (rows >= T_ are masked in the step)
      char* lb = smem + slot * BUF;
#pragma unroll
      for (int j = 0; j < PPW; ++j) {
        const int P = (w + 4 * j) * 64 + lane;
        const int r = P / CH, pc = P % CH;
        int rc;
        if constexpr (DUAL) rc = pc ^ dual_f<HD>(r);
        else if constexpr (HD == 128) rc = pc ^ (r & 15);
        else rc = pc ^ ((r >> 1) & 7);
        const int c64 = (pc >> 2) ^ (HD == 128 ? (r & 3) : ((r >> 1) & 1));
        const int tc = c64 * 4 + (pc & 3);
        const uint32_t pd = (w + 4 * j) * 1024;
        const int rr = min(q0 + r, T_ - 1);
        glds16(qb_ + (long)rr * rs + rc * 8, lb + pd);
        if constexpr (!DUAL) glds16(qb_ + (long)rr * rs + tc * 8, lb + IQT + pd);
        glds16(ob_ + (long)rr * ors + rc * 8, lb + IOR + pd);
        if constexpr (!DUAL) glds16(ob_ + (long)rr * ors + tc * 8, lb + IOT + pd);
      }
    }
    glds4(stat_src + min(q0 + l32, T_ - 1), smem + slot * BUF + ISTAT + w * 256);
    if constexpr (MASK)  // words (q0 .. q0+31, this wave's key word); the upper half duplicates
      glds4(kmask + (long)(b * H + h) * kw_row + (long)min(kw0 >> 5, (T_ - 1) >> 5) * T_ + min(q0 + l32, T_ - 1),
            smem + slot * BUF + IMASK + w * 256);
  };
  // wait until step i+1's DMA landed, leaving the later issued steps (up to NBUF-2) in flight
  auto ring_wait = [&](int i, int nsteps) {
    if constexpr (NBUF == 4) {
      if (i + 3 < nsteps) wait_vm<2 * NPW>(); else if (i + 2 < nsteps) wait_vm<NPW>(); else wait_vm0();
    } else if constexpr (NBUF == 3) {
      if (i + 2 < nsteps) wait_vm<NPW>(); else wait_vm0();
    } else {
      wait_vm0();
    }
    __builtin_amdgcn_s_barrier();
  };

  const int qstart = causal ? k0 : 0;
  const int nsteps = qstart < T_ ? (T_ - qstart + BWD_BQ - 1) / BWD_BQ : 0;
#pragma unroll
  for (int j = 0; j < NBUF - 1; ++j)
    if (j < nsteps) issue(qstart + j * BWD_BQ, j);
  // step 0 landed; steps 1 .. min(nsteps, NBUF-1)-1 may still fly
  if constexpr (NBUF == 4) {
    if (nsteps > 2) wait_vm<2 * NPW>(); else if (nsteps > 1) wait_vm<NPW>(); else wait_vm0();
  } else if constexpr (NBUF == 3) {
    if (nsteps > 1) wait_vm<NPW>(); else wait_vm0();
  } else {
    wait_vm0();
  }
  __builtin_amdgcn_s_barrier();
  // Steps before this wave's first active one (causal: the wave's keys are above them) only
  // keep the DMA ring and the barriers going; the compute loop after them runs the MFMAs on
  // every step, so dK/dV stay in the same accumulator registers across iterations.
  const int first = kw0 >= T_ ? nsteps : (causal ? min(w, nsteps) : 0);
  int slot = 0, i = 0;
  for (; i < first; ++i) {
    if (i + NBUF - 1 < nsteps) issue(qstart + (i + NBUF - 1) * BWD_BQ, slot == 0 ? NBUF - 1 : slot - 1);
    ring_wait(i, nsteps);
    slot = slot == NBUF - 1 ? 0 : slot + 1;
  }
  for (; i < nsteps; ++i) {
    const int q0 = qstart + i * BWD_BQ;
    if (i + NBUF - 1 < nsteps) issue(q0 + (NBUF - 1) * BWD_BQ, slot == 0 ? NBUF - 1 : slot - 1);
    const char* S = smem + slot * BUF;
    // per-lane LDS offsets, recomputed each step from an opaque copy of the lane id (a few
    // VALU) instead of being held in VGPRs across the loop
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int hh_ = ln >> 5, l32_ = ln & 31, gi = ln & 15;
    const int gl = (gi >> 4) & 1;  // always 0 for gi < 16; kept for the transposed-read form
    (void)gl;
    const int qrow = gi >> 2, pcol = gi & 3, glb = (ln >> 4) & 1;
    // wave-uniform: the diagonal step or a sequence tail needs masking
    const bool edge = (causal && i == first) || q0 + BWD_BQ > T_ || kw0 + 32 > T_;
    {
      f32x16 sacc = f32x16{}, dpacc = f32x16{};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int ro = DUAL ? dual_off<HD>(l32_, kk * 2 + hh_) : r_off<HD>(l32_, kk * 2 + hh_);
        sacc = MFb<T>::mma(*reinterpret_cast<const v8*>(S + ro), kf[kk], sacc);
        v8 vk;
        if constexpr (VLDS) vk = *reinterpret_cast<const v8*>(smem + VOFF + w * 32 * ROWB + r_off<HD>(l32_, kk * 2 + hh_));
        else vk = vf[kk];
        dpacc = MFb<T>::mma(*reinterpret_cast<const v8*>(S + IOR + ro), vk, dpacc);
      }
      // rows of this lane's accumulator registers: q = q0 + 4hh + off, off = (r&3) + 8(r>>2);
      // visible iff lo <= off <= hi (causal: q >= key; q < T; key < T)
      if (edge) {
        // (the empty volatile asm keeps hipcc from if-converting this rare branch into
        // per-step selects on every element)
        asm volatile("" ::: "memory");
        const int qb0 = q0 + 4 * hh;
        const int lo = causal ? mykey - qb0 : -(1 << 30);
        const int hi = mykey < T_ ? T_ - 1 - qb0 : -(1 << 30);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int off = (r & 3) + 8 * (r >> 2);
          if (off < lo || off > hi) sacc[r] = -INFINITY;
        }
      }
      const float* LS = reinterpret_cast<const float*>(S + ISTAT + w * 256);
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const f32x4 L4 = *reinterpret_cast<const f32x4*>(LS + 8 * gq + 4 * hh_);
        const f32x4 D4 = *reinterpret_cast<const f32x4*>(LS + 32 + 8 * gq + 4 * hh_);
        uint4 M4 = {0u, 0u, 0u, 0u};
        if constexpr (MASK) M4 = *reinterpret_cast<const uint4*>(S + IMASK + w * 256 + 4 * (8 * gq + 4 * hh_));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * gq + j;
          const float p = __builtin_amdgcn_exp2f(fmaf(sacc[r], c, -L4[j]));
          float dp = dpacc[r], pd = p;
          if constexpr (DROP) {
            bool keep;
            if constexpr (MASK) {
              const uint32_t mw = j == 0 ? M4.x : j == 1 ? M4.y : j == 2 ? M4.z : M4.w;
              keep = (mw >> l32_) & 1u;
            } else {
              const int q = q0 + 8 * gq + 4 * hh + j;
              keep = ds.bits16(dslab + (uint64_t)q * T_ + mykey) >= thr;
            }
            pd = keep ? p * inv_keep : 0.f;
            dp = keep ? dp * inv_keep : 0.f;
          }
          sacc[r] = pd;
          dpacc[r] = p * (dp - D4[j]);
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
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          int olo, ohi;
          if constexpr (DUAL) {
            // lane 4q+p of a 16-lane group: row 4hh+q (+8), columns dt*32 + glb*16 + 4p .. +3
            const int row = 4 * hh_ + qrow + s2 * 16, ch = dt * 4 + glb * 2 + (pcol >> 1);
            olo = dual_off<HD>(row, ch) + 8 * (pcol & 1);
            ohi = dual_off<HD>(row + 8, ch) + 8 * (pcol & 1);
          } else {
            olo = t_off<HD>(4 * hh_ + qrow, dt * 32 + glb * 16 + pcol * 4) + s2 * 16 * ROWB;
            ohi = olo + 8 * ROWB;
          }
          const v8 ao = tr8<v8>(S + IOT, olo, ohi);
          dv[dt] = MFb<T>::mma(ao, pf, dv[dt]);
          const v8 aq = tr8<v8>(S + IQT, olo, ohi);
          dk[dt] = MFb<T>::mma(aq, df, dk[dt]);
        }
      }
    }
    ring_wait(i, nsteps);
    slot = slot == NBUF - 1 ? 0 : slot + 1;
  }

  }  // heads

  // ---- MHA / fused GQA: write bf16 dK/dV straight into dqkv; else per-head fp32 partials
  const int h = h_first;
  if (mykey < T_ && (FUSEG || H == G)) {
    T* pk = dqkv + ((long)b * T_ + mykey) * rs + (long)(H + g) * HD;
    T* pv = dqkv + ((long)b * T_ + mykey) * rs + (long)(H + G + g) * HD;
    if (rcos) {  // the backward of the forward's RoPE on K, applied to dK before it is stored
#pragma unroll
      for (int dt = 0; dt < DT / 2; ++dt) rope_bwd_store<T, HD>(dk[dt], dk[dt + DT / 2], scale, hh, mykey, dt * 32, rcos, rsin, pk);
    } else {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int gq = 0; gq < 4; gq += 2) {
          const uint32_t a[2] = {pk2<T>(dk[dt][4 * gq] * scale, dk[dt][4 * gq + 1] * scale),
                                 pk2<T>(dk[dt][4 * gq + 2] * scale, dk[dt][4 * gq + 3] * scale)};
          const uint32_t c[2] = {pk2<T>(dk[dt][4 * gq + 4] * scale, dk[dt][4 * gq + 5] * scale),
                                 pk2<T>(dk[dt][4 * gq + 6] * scale, dk[dt][4 * gq + 7] * scale)};
          store16_pair<T>(pk + dt * 32 + 8 * gq + 8 * hh, a, c);
        }
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; gq += 2) {
        const uint32_t a[2] = {pk2<T>(dv[dt][4 * gq], dv[dt][4 * gq + 1]), pk2<T>(dv[dt][4 * gq + 2], dv[dt][4 * gq + 3])};
        const uint32_t c[2] = {pk2<T>(dv[dt][4 * gq + 4], dv[dt][4 * gq + 5]), pk2<T>(dv[dt][4 * gq + 6], dv[dt][4 * gq + 7])};
        store16_pair<T>(pv + dt * 32 + 8 * gq + 8 * hh, a, c);
      }
  } else if (mykey < T_) {
    const long BT = (long)B_ * T_;
    float* pk = dkv_part + ((long)b * T_ + mykey) * ors + (long)h * HD;
    float* pv = pk + BT * ors;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d0 = dt * 32 + 8 * gq + 4 * hh;
        *reinterpret_cast<f32x4*>(pk + d0) = f32x4{dk[dt][4 * gq] * scale, dk[dt][4 * gq + 1] * scale,
                                                   dk[dt][4 * gq + 2] * scale, dk[dt][4 * gq + 3] * scale};
        *reinterpret_cast<f32x4*>(pv + d0) = f32x4{dv[dt][4 * gq], dv[dt][4 * gq + 1], dv[dt][4 * gq + 2], dv[dt][4 * gq + 3]};
      }
  }
}

// ---------------------------------------------------------------------------------------
// dQ kernel (forward-shaped): 4 waves x 32 queries of head h; key tiles of 64 by saddr DMA
// (3-slot ring, prefetch distance 2) into three images per slot: K rows (S^T = K Q^T),
// K transposed (dQ^T += K^T dS^T), V rows (dP^T = V dO^T).  The query is the lane column, so
// lse / delta are per-lane scalars; 1/sqrt(d) is applied once to the final dQ.
constexpr int DQ_BQ = 128;
template <int HD, int BK, bool MASK = false> constexpr int dq_buf_bytes() {
  return 3 * BK * HD * 2 + (MASK ? 4 * 256 : 0);
}

// MASK (with DROP): keep bits from the forward's keep mask (one 4-byte DMA per wave and tile:
// the words of the wave's 32 queries for each 32-key sub-tile) instead of the counter hash.
template <typename T, int HD, bool DROP, int DQ_BK, int NBUF, int OCC, bool MASK = false>
__global__ __launch_bounds__(256, OCC) void attn_bwd_dq_k(const T* __restrict__ qkv, const T* __restrict__ out,
                                                        const T* __restrict__ dout,
                                                        const float* __restrict__ lse,
                                                        float* __restrict__ delta, T* __restrict__ dqkv,
                                                        int T_, int H, int G, int B_, bool causal, uint32_t thr,
                                                        float inv_keep, uint64_t seed, uint64_t doff,
                                                        const uint32_t* __restrict__ kmask,
                                                        const float* __restrict__ rcos,
                                                        const float* __restrict__ rsin, int xmap) {
  typedef typename MFb<T>::v8 v8;
  constexpr int KK = HD / 16, DT = HD / 32, CH = HD / 8, ROWB = HD * 2;
  constexpr int IMG = DQ_BK * ROWB;             // bytes of one [BK][HD] image
  constexpr int LD = DQ_BK * CH / 256;          // 1-KiB pieces per wave per image
  constexpr int NKT = DQ_BK / 32;               // 32-key MFMA tiles per step
  constexpr int BUF = dq_buf_bytes<HD, DQ_BK, MASK>();
  static_assert(NBUF == 2 || NBUF == 3, "ring depth");
  static_assert(!MASK || DROP, "keep mask only with dropout");
  static_assert(DQ_BK / 32 <= 2, "mask words: one lane half per 32-key sub-tile");
  constexpr int NPW = 3 * LD + (MASK ? 1 : 0);  // DMA instructions per wave per step
  constexpr int MOFF = 3 * IMG;                 // per-wave keep-mask words (MASK)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // heaviest (last, for causal) query block first; the query heads of one kv head on one XCD
  // (xmap 1, common.h attn_wg_order: they share the K/V stream)
  const int nqb = (T_ + DQ_BQ - 1) / DQ_BQ;
  const int lin = blockIdx.x, nbh = H * B_;
  int qbi, bh;
  attn_wg_order(lin, nbh, H / G, xmap, qbi, bh);
  const int qb = causal ? nqb - 1 - qbi : qbi;
  const int h = bh % H, b = bh / H;
  const int g = h / (H / G);
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gi = lane & 15, gl = (lane >> 4) & 1, qrow = gi >> 2, pcol = gi & 3;
  const long rs = (long)(H + 2 * G) * HD;
  const long ors = (long)H * HD;
  const T* kb_ = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const T* vb_ = qkv + (long)b * T_ * rs + (long)(H + G + g) * HD;
  const int q0 = qb * DQ_BQ;
  const int wq_lo = q0 + w * 32, wq_hi = wq_lo + 31;
  const int qi = wq_lo + l32;
  const int qc = qi < T_ ? qi : T_ - 1;
  const float scale = rsqrtf((float)HD), c = scale * kLog2eB;
  DropSlab ds;
  uint64_t dslab = 0;
  if constexpr (DROP) {
    dslab = doff + (uint64_t)(b * H + h) * T_ * T_;
    ds.init(seed, dslab);
  }
  const bool dpair = ((doff | (uint64_t)T_) & 1) == 0;

  v8 qf[KK], of[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    qf[kk] = *reinterpret_cast<const v8*>(qkv + ((long)b * T_ + qc) * rs + (long)h * HD + kk * 16 + hh * 8);
    of[kk] = *reinterpret_cast<const v8*>(dout + ((long)b * T_ + qc) * ors + (long)h * HD + kk * 16 + hh * 8);
  }
  const float L = lse[((long)b * H + h) * T_ + qc];
  // delta = rowsum(dO * O): this lane holds half of the row (elements 16kk + 8hh + 0..7)
  float D;
  {
    float part = 0.f;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const v8 ov = *reinterpret_cast<const v8*>(out + ((long)b * T_ + qc) * ors + (long)h * HD + kk * 16 + hh * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) part += (float)ov[j] * (float)of[kk][j];
    }
    D = part + __shfl_xor(part, 32, 64);
    if (hh == 0 && qi < T_) delta[((long)b * H + h) * T_ + qi] = D;
  }
  {
    float lt = L, dt_ = D;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) asm volatile("" ::"v"(qf[kk]), "v"(of[kk]));
    asm volatile("" ::"v"(lt), "v"(dt_));
  }
  f32x16 dq[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dq[i] = f32x16{};

  int roff[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) roff[kk] = r_off<HD>(l32, kk * 2 + hh);
  int troff[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) troff[dt] = t_off<HD>(4 * hh + qrow, dt * 32 + gl * 16 + pcol * 4);
  uint32_t roffg[LD], toffg[LD];
  int prow[LD], prc[LD], ptc[LD];
#pragma unroll
  for (int i = 0; i < LD; ++i) {
    const int P = (w * LD + i) * 64 + lane;
    const int r = P / CH, pc = P % CH;
    int rc;
    if constexpr (HD == 128) rc = pc ^ (r & 15); else rc = pc ^ ((r >> 1) & 7);
    const int c64 = (pc >> 2) ^ (HD == 128 ? (r & 3) : ((r >> 1) & 1));
    const int tc = c64 * 4 + (pc & 3);
    prow[i] = r; prc[i] = rc; ptc[i] = tc;
    roffg[i] = (uint32_t)(r * rs * 2 + rc * 16);
    toffg[i] = (uint32_t)(r * rs * 2 + tc * 16);
  }
  const uint32_t smem_u = lds_u32(smem);

  const long kw_row = (long)((T_ + 31) / 32) * T_;  // keep-mask words per (b, h)
  auto issue = [&](int t, int slot) {
    const int k0 = t * DQ_BK;
    const uint32_t base = smem_u + slot * BUF;
    if constexpr (MASK) {  // lane half kt: words (wave's queries, key word t*NKT + kt)
      const int kw = min(t * NKT + (NKT == 2 ? hh : 0), (T_ - 1) >> 5);
      glds4(kmask + (long)(b * H + h) * kw_row + (long)kw * T_ + qc, smem + slot * BUF + MOFF + w * 256);
    }
    if (k0 + DQ_BK <= T_) {
      const void* ks = sgpr_ptr(kb_ + (long)k0 * rs);
      const void* vs = sgpr_ptr(vb_ + (long)k0 * rs);
#pragma unroll
      for (int i = 0; i < LD; ++i) {
        const uint32_t pd = (w * LD + i) * 1024;
        glds16s(ks, roffg[i], base + pd);
        glds16s(ks, toffg[i], base + IMG + pd);
        glds16s(vs, roffg[i], base + 2 * IMG + pd);
      }
    } else {  // sequence tail: clamp rows (keys >= T_ are masked)
      char* lb = smem + slot * BUF;
#pragma unroll
      for (int i = 0; i < LD; ++i) {
        const int pd = (w * LD + i) * 1024;
        const int key = min(k0 + prow[i], T_ - 1);
        glds16(kb_ + (long)key * rs + prc[i] * 8, lb + pd);
        glds16(kb_ + (long)key * rs + ptc[i] * 8, lb + IMG + pd);
        glds16(vb_ + (long)key * rs + prc[i] * 8, lb + 2 * IMG + pd);
      }
    }
  };

  const int kend = causal ? min(T_, q0 + DQ_BQ) : T_;
  const int ntiles = (kend + DQ_BK - 1) / DQ_BK;
  // tiles this wave computes: all up to the one holding its last query (causal)
  const int nact = wq_lo >= T_ ? 0 : (causal ? min(ntiles, wq_hi / DQ_BK + 1) : ntiles);
  auto ring_wait = [&](int t) {
    if constexpr (NBUF == 3) {
      if (t + 2 < ntiles) wait_vm<NPW>(); else wait_vm0();
    } else {
      wait_vm0();
    }
    __builtin_amdgcn_s_barrier();
  };
#pragma unroll
  for (int j = 0; j < NBUF - 1; ++j)
    if (j < ntiles) issue(j, j);
  if constexpr (NBUF == 3) {
    if (ntiles > 1) wait_vm<NPW>(); else wait_vm0();
  } else {
    wait_vm0();
  }
  __builtin_amdgcn_s_barrier();
  int slot = 0, t = 0;
  for (; t < nact; ++t) {
    if (t + NBUF - 1 < ntiles) issue(t + NBUF - 1, slot == 0 ? NBUF - 1 : slot - 1);
    const int k0 = t * DQ_BK;
    const char* KR = smem + slot * BUF;
    const char* KT = KR + IMG;
    const char* VR = KR + 2 * IMG;
    f32x16 sc[NKT], dp[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      sc[kt] = f32x16{};
      dp[kt] = f32x16{};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int off = kt * 32 * ROWB + roff[kk];
        sc[kt] = MFb<T>::mma(*reinterpret_cast<const v8*>(KR + off), qf[kk], sc[kt]);
        dp[kt] = MFb<T>::mma(*reinterpret_cast<const v8*>(VR + off), of[kk], dp[kt]);
      }
    }
    // keys of this lane's accumulator rows: k0 + 32kt + (r&3) + 8(r>>2) + 4hh
    const bool edge = (causal && k0 + DQ_BK - 1 > wq_lo) || k0 + DQ_BK > T_ || wq_hi >= T_;
    if (edge) {
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if ((causal && key > qi) || key >= T_ || qi >= T_) sc[kt][r] = -INFINITY;
        }
    }
    if constexpr (MASK) {
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const uint32_t mw = *reinterpret_cast<const uint32_t*>(KR + MOFF + w * 256 + 4 * (kt * 32 + l32)) >> (4 * hh);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          dp[kt][r] = ((mw >> ((r & 3) + 8 * (r >> 2))) & 1u) ? dp[kt][r] * inv_keep : 0.f;
      }
    } else if constexpr (DROP) {
      const uint64_t rowbase = dslab + (uint64_t)qi * T_;
      if (dpair) {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const uint32_t hv = ds.pair_hash((rowbase + key) >> 1);
            dp[kt][r] = (hv & 0xFFFFu) >= thr ? dp[kt][r] * inv_keep : 0.f;
            dp[kt][r + 1] = (hv >> 16) >= thr ? dp[kt][r + 1] * inv_keep : 0.f;
          }
      } else {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            dp[kt][r] = ds.bits16(rowbase + key) >= thr ? dp[kt][r] * inv_keep : 0.f;
          }
      }
    }
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sc[kt][r], c, -L));
        sc[kt][r] = p * (dp[kt][r] - D);
      }
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        v8 df;
        {
          uint32_t u[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) u[j] = pk2<T>(sc[kt][8 * s2 + 2 * j], sc[kt][8 * s2 + 2 * j + 1]);
          __builtin_memcpy(&df, u, 16);
        }
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int o = troff[dt] + (kt * 32 + s2 * 16) * ROWB;
          const v8 a = tr8<v8>(KT, o, o + 8 * ROWB);
          dq[dt] = MFb<T>::mma(a, df, dq[dt]);
        }
      }
    ring_wait(t);
    slot = slot == NBUF - 1 ? 0 : slot + 1;
  }
  for (; t < ntiles; ++t) {  // this wave is done; keep the ring and barriers going
    if (t + NBUF - 1 < ntiles) issue(t + NBUF - 1, slot == 0 ? NBUF - 1 : slot - 1);
    ring_wait(t);
    slot = slot == NBUF - 1 ? 0 : slot + 1;
  }
  if (qi < T_) {
    T* row = dqkv + ((long)b * T_ + qi) * rs + (long)h * HD;
    if (rcos) {  // the backward of the forward's RoPE on Q, applied to dQ before it is stored
#pragma unroll
      for (int dt = 0; dt < DT / 2; ++dt) rope_bwd_store<T, HD>(dq[dt], dq[dt + DT / 2], scale, hh, qi, dt * 32, rcos, rsin, row);
      return;
    }
    // 16-B stores (store16_pair)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; gq += 2) {
        const uint32_t a[2] = {pk2<T>(dq[dt][4 * gq] * scale, dq[dt][4 * gq + 1] * scale),
                               pk2<T>(dq[dt][4 * gq + 2] * scale, dq[dt][4 * gq + 3] * scale)};
        const uint32_t c[2] = {pk2<T>(dq[dt][4 * gq + 4] * scale, dq[dt][4 * gq + 5] * scale),
                               pk2<T>(dq[dt][4 * gq + 6] * scale, dq[dt][4 * gq + 7] * scale)};
        store16_pair<T>(row + dt * 32 + 8 * gq + 8 * hh, a, c);
      }
  }
}

// GQA: dqkv[:, k/v part] = bf16(sum over the H/G query heads of each kv group)
// With rcos: the inverse RoPE on dK as well (the thread of the first-half chunk d also sums the
// chunk d + HD/2 and writes both; second-half threads of K have nothing to do).
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_kv_reduce_k(const float* __restrict__ dkv_part, T* __restrict__ dqkv,
                                                            long BT, int H, int G, int HD, int T_,
                                                            const float* __restrict__ rcos,
                                                            const float* __restrict__ rsin) {
  const int rep = H / G, half = HD / 2;
  const long rs = (long)(H + 2 * G) * HD;
  const long per_row = 2L * G * HD / 4;
  const long total = BT * per_row;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long row = i / per_row;
    const int kvcol = (int)(i - row * per_row) * 4;  // in [0, 2*G*HD)
    const int which = kvcol / (G * HD);
    const int gg = (kvcol % (G * HD)) / HD, d = kvcol % HD;
    const bool rot = rcos && which == 0;
    if (rot && d >= half) continue;
    const float* src = dkv_part + (long)which * BT * H * HD + row * H * HD;
    float v[4] = {0.f, 0.f, 0.f, 0.f}, w[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < rep; ++r) {
      const float4 x = *reinterpret_cast<const float4*>(src + (long)(gg * rep + r) * HD + d);
      v[0] += x.x; v[1] += x.y; v[2] += x.z; v[3] += x.w;
      if (rot) {
        const float4 y = *reinterpret_cast<const float4*>(src + (long)(gg * rep + r) * HD + d + half);
        w[0] += y.x; w[1] += y.y; w[2] += y.z; w[3] += y.w;
      }
    }
    T* dst = dqkv + row * rs + (long)H * HD + kvcol;
    if (rot) {
      const int pos = (int)(row % T_);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = rcos[(long)pos * half + d + j], sn = rsin[(long)pos * half + d + j];
        dst[j] = from_f<T>(v[j] * c + w[j] * sn);
        dst[j + half] = from_f<T>(w[j] * c - v[j] * sn);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = from_f<T>(v[j]);
    }
  }
}

// GQA heads of a kv head fused into one dK/dV workgroup (no per-head fp32 partials, no
// reduction pass) when the fused grid still has >= 4 workgroups per CU (Llama-3-8B B=24
// 1.51 -> 1.12 ms); below that the per-head grid wins (B=4: 256 fused workgroups, 0.25 ms unfused
// vs 0.35 fused).  Dropped variants (3-slot ring at one workgroup per CU, 64-key dQ tiles) are
// in profiles/r2_kernel_experiments.md.
static bool fuse_gqa_heads(int B, int T_, int H, int G) {
  if (H == G) return false;
  const long nkb = (T_ + BWD_BKV - 1) / BWD_BKV;
  return nkb * G * (long)B >= 1024;
}

bool attn_bwd_kv_partials(int B, int T_, int H, int G) { return H != G && !fuse_gqa_heads(B, T_, H, G); }

// launch helpers: one instantiation per (ring, occupancy, fused heads, dual images) and per
// dropout form (none / counter hash / forward keep mask)
struct BwdArgs {
  const void *qkv, *o, *dout;
  const float* lse;
  float *delta, *dkv_part;
  void* dqkv;
  int T_, H, G, B;
  bool causal;
  uint32_t thr;
  float ik;
  uint64_t seed, offset;
  const uint32_t* kmask;
  const float *rcos, *rsin;
  hipStream_t s;
  int xmap_q, xmap_kv;  // attn_wg_order modes of the dQ / dK-dV grids
};
template <typename TT, int HDD, bool DROP, int BK, int NB, int OC, bool MASK>
static void launch_dq1(const BwdArgs& a, dim3 grid) {
  constexpr int lds = NB * dq_buf_bytes<HDD, BK, MASK>();
  hipLaunchKernelGGL((attn_bwd_dq_k<TT, HDD, DROP, BK, NB, OC, MASK>), grid, dim3(256), lds, a.s, (const TT*)a.qkv, (const TT*)a.o, (const TT*)a.dout, a.lse, a.delta, (TT*)a.dqkv, a.T_, a.H,
                     a.G, a.B, a.causal, a.thr, a.ik, a.seed, a.offset, a.kmask, a.rcos, a.rsin, a.xmap_q);
}
template <typename TT, int HDD, int BK, int NB, int OC>
static void launch_dq(const BwdArgs& a, bool drop, dim3 grid) {
  if (drop && a.kmask) launch_dq1<TT, HDD, true, BK, NB, OC, true>(a, grid);
  else if (drop) launch_dq1<TT, HDD, true, BK, NB, OC, false>(a, grid);
  else launch_dq1<TT, HDD, false, BK, NB, OC, false>(a, grid);
}
template <typename TT, int HDD, bool DROP, int NB, int OC, bool FG, bool DU, bool MASK, bool VL>
static void launch_kv1(const BwdArgs& a, dim3 grid) {
  constexpr int lds = NB * dkdv_buf_bytes<HDD, DU, MASK>() + (VL ? BWD_BKV * HDD * 2 : 0);
  hipLaunchKernelGGL((attn_bwd_mfma_k<TT, HDD, DROP, NB, OC, FG, DU, MASK, VL>), grid, dim3(256), lds, a.s, (const TT*)a.qkv, (const TT*)a.dout, a.lse, a.delta,
                     (TT*)a.dqkv, a.dkv_part, a.T_, a.H, a.G, a.B, a.causal, a.thr, a.ik, a.seed, a.offset, a.kmask,
                     a.rcos, a.rsin, a.xmap_kv);
}
template <typename TT, int HDD, int NB, int OC, bool FG, bool DU, bool VL = false>
static void launch_kv(const BwdArgs& a, bool drop, dim3 grid) {
  if (drop && a.kmask) launch_kv1<TT, HDD, true, NB, OC, FG, DU, true, VL>(a, grid);
  else if (drop) launch_kv1<TT, HDD, true, NB, OC, FG, DU, false, VL>(a, grid);
  else launch_kv1<TT, HDD, false, NB, OC, FG, DU, false, VL>(a, grid);
}
// dQ: 32-key tiles, 3-slot ring, 2 workgroups per CU.  dK/dV: hd 128 -> one dual-use LDS image
// per Q / dO tile, V fragments in LDS, 2-slot ring (Llama-3-8B B=24 1.158 -> 1.009 ms); hd 64 ->
// dual images only with the forward's dropout keep mask (GPT2-774M B=24 0.430 -> 0.420 ms; they
// lose without dropout or with fused GQA heads: 0.367 -> 0.376, Llama-3.2-1B 0.575 -> 0.602 ms,
// profiles/r2_attn_hd64_dual.md), 4-slot ring; else separate row / transposed images, 2-slot ring
template <typename TT, int HDD>
static void launch_bwd(const BwdArgs& a, bool drop, bool fuseg, dim3 grid_q, dim3 grid_kv) {
  launch_dq<TT, HDD, 32, 3, 2>(a, drop, grid_q);
  if constexpr (HDD == 128) {
    if (fuseg) launch_kv<TT, HDD, 2, 2, true, true, true>(a, drop, grid_kv);
    else launch_kv<TT, HDD, 2, 2, false, true, true>(a, drop, grid_kv);
  } else {
    // keep-mask dual-image variant at a launch bound of 3 workgroups per CU (168 VGPRs, 3 waves
    // per SIMD instead of 2 at 170): GPT2-774M B=64 backward 1.260 -> 1.195 ms, B=24 0.448 ->
    // 0.417 (profiles/r6/attn/occ_ab.jsonl)
    if (drop && a.kmask && !fuseg) launch_kv<TT, HDD, 4, 3, false, true>(a, drop, grid_kv);
    else if (fuseg) launch_kv<TT, HDD, 2, 2, true, false>(a, drop, grid_kv);
    else launch_kv<TT, HDD, 2, 2, false, false>(a, drop, grid_kv);
  }
}

void attn_bwd_mfma(DType dt, const void* qkv, const void* o, const float* lse, const void* dout, void* dqkv,
                   float* delta, float* dq_acc, float* dkv_part, int B, int T_, int H, int G, int hd, bool causal,
                   float p, uint64_t seed, uint64_t offset, const uint32_t* keep_mask, const float* rcos,
                   const float* rsin, hipStream_t s) {
  (void)dq_acc;
  const int nkb = (T_ + BWD_BKV - 1) / BWD_BKV;
  const bool fuseg = fuse_gqa_heads(B, T_, H, G);
  dim3 grid_kv(nkb * (fuseg ? G : H) * B), grid_q(((T_ + DQ_BQ - 1) / DQ_BQ) * H * B);
  const bool drop = p > 0.f;
  const int xq = attn_xcd_order_ok(B * H, H / G) ? 1 : 0;
  const int xkv = attn_xcd_order_ok((fuseg ? G : H) * B, 1) ? 1 : 0;
  const BwdArgs a{qkv, o, dout, lse, delta, dkv_part, dqkv, T_, H, G, B, causal, drop_threshold16(p),
                  drop_inv_keep(p), seed, offset, drop ? keep_mask : nullptr, rcos, rsin, s, xq, xkv};
  if (dt == DType::BF16) {
    if (hd == 128) launch_bwd<bf16_t, 128>(a, drop, fuseg, grid_q, grid_kv);
    else launch_bwd<bf16_t, 64>(a, drop, fuseg, grid_q, grid_kv);
  } else {
    if (hd == 128) launch_bwd<f16_t, 128>(a, drop, fuseg, grid_q, grid_kv);
    else launch_bwd<f16_t, 64>(a, drop, fuseg, grid_q, grid_kv);
  }
  if (H != G && !fuseg) {
    const long BT = (long)B * T_;
    const long groups = BT * 2L * G * hd / 4;
    const int fg = (int)((groups + 255) / 256 < 4096 ? (groups + 255) / 256 : 4096);
    BLLM_DISPATCH(dt, TT, {
      hipLaunchKernelGGL(attn_bwd_kv_reduce_k<TT>, dim3(fg), dim3(256), 0, s, dkv_part, (TT*)dqkv, BT, H, G, hd, T_,
                         rcos, rsin);
    });
  }
}

}  // namespace bllm
