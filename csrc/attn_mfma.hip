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
// Workgroup = 4 waves; each wave owns one 32-query block (128 queries per workgroup; two blocks
// per wave, which halves the LDS reads per FLOP, measured slower on every shape:
// profiles/r3/attn_fwd_qb2.md -- the per-query arrays below keep a block index for that layout).
// K/V tiles of 64 keys, register DMA (global_load_lds) of tile t+1 under the MFMAs of tile t,
// double-buffered LDS.  GQA reads kv head h / (H/G)
// directly; causal tiles above the diagonal are skipped; q-blocks are launched
// heaviest-first.  LDS images are XOR-swizzled: K in 16-B chunks (conflict-free
// ds_read_b128 row reads), V in 64-B chunks (conflict-free transposed reads).
// Attention-probability dropout (GPT-2) uses the stateless counter hash of common.h.
#include <float.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>
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
constexpr float kRescaleThr = 8.f;  // deferred online-softmax rescale threshold (log2 units)
constexpr int FWD_BQ = 128;  // queries per workgroup per q-block of each wave (x QB)
// keys per tile (FWD_BK), LDS ring depth and workgroups per CU are template parameters

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

// two floats -> packed pair (one v_cvt_pk_bf16_f32 for bf16)
template <typename T> __device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef T t2 __attribute__((ext_vector_type(2)));
  const t2 v = __builtin_convertvector((f2{a, b}), t2);
  uint32_t u;
  __builtin_memcpy(&u, &v, 4);
  return u;
}

// Per 64-key tile and wave: 32 MFMAs, 16 b128 + 32 tr_b64 LDS reads at loop-invariant
// per-lane offsets, 2x(LD) saddr DMA issues with precomputed per-lane source offsets, and
// ~130 VALU of online softmax (scale folded into the exp2 FMA; the O rescale is skipped when
// no lane's running max moved, which is the common case after the first tiles).  The LDS
// fragment reads run one MFMA step ahead (QK^T: both 32-key sub-tiles' next K fragments before
// this step's pair of MFMAs, pinned by sched_barrier; PV: the next V^T fragment before each
// MFMA): hipcc's own schedule waited on every read right before its MFMA (round 6, headline
// forward +1.5 % same process, profiles/r6/attn/).
template <typename T, int HD, bool DROP, int FWD_BK, int NBUF, int OCC>
__global__ __launch_bounds__(256, OCC) void attn_fwd_mfma_k(const T* __restrict__ qkv, T* __restrict__ out,
                                                          float* __restrict__ lse, int T_, int H, int G, int B_,
                                                          bool causal, uint32_t thr, float inv_keep, uint64_t seed,
                                                          uint64_t doff, uint32_t* __restrict__ kmask, bool xmap) {
  typedef typename MF<T>::v8 v8;
  constexpr int KK = HD / 16;               // k-steps of the QK^T product
  constexpr int DT = HD / 32;               // 32-row tiles of O^T
  constexpr int CH = HD / 8;                // 16-B chunks per K/V row
  constexpr int ROWB = HD * 2;
  constexpr int TILE_B = FWD_BK * ROWB;     // bytes per K (or V) tile
  constexpr int LD = FWD_BK * CH / 256;     // 1-KiB pieces per wave per tile (K and V each)
  constexpr int NPW = 2 * LD;
  constexpr int NKT = FWD_BK / 32;          // 32-key MFMA tiles per step
  constexpr int QB = 1;                     // 32-query blocks per wave
  constexpr int WQ = 32 * QB;               // queries per wave
  constexpr int BQ = FWD_BQ * QB;           // queries per workgroup
  static_assert(NBUF == 2 || NBUF == 3, "ring depth");

  extern __shared__ __attribute__((aligned(16))) char smem[];

  // heaviest (latest, for causal) q-blocks first over the whole grid; the q-blocks of one
  // (b, h) share lin % 8 (one XCD / L2 for their common K/V stream)
  const int nqb = (T_ + BQ - 1) / BQ;
  const int lin = blockIdx.x, nbh = H * B_;
  int qbi, h, b;
  if (xmap) {
    // XCD-aware order (B G % 8 == 0): workgroup lin runs on XCD lin % 8 (round-robin dispatch);
    // XCD x takes the (batch, kv-head) groups bg with bg % 8 == x, and its k-th workgroup is
    // (q-block k / per_qb heaviest first, group, query head of the group): the query heads that
    // share one K/V stream run back to back on one L2
    const int x = lin & 7, k = lin >> 3, hpg = H / G;
    const int per_qb = (B_ * G / 8) * hpg;
    qbi = k / per_qb;
    const int rem = k - qbi * per_qb, bgl = rem / hpg;
    const int bg = bgl * 8 + x;
    b = bg / G;
    h = (bg - b * G) * hpg + (rem - bgl * hpg);
  } else {
    qbi = lin / nbh;
    const int bh = lin - qbi * nbh;
    h = bh % H;
    b = bh / H;
  }
  const int qb = causal ? nqb - 1 - qbi : qbi;
  const int g = h / (H / G);
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gi = lane & 15, gl = (lane >> 4) & 1, qrow = gi >> 2, pcol = gi & 3;
  const long rs = (long)(H + 2 * G) * HD;
  const T* qbase = qkv + (long)b * T_ * rs + (long)h * HD;
  const T* kbase = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const T* vbase = qkv + (long)b * T_ * rs + (long)(H + G + g) * HD;
  const int q0 = qb * BQ;
  const int wq_lo = q0 + w * WQ, wq_hi = wq_lo + WQ - 1;  // this wave's query range
  int qi[QB];                                             // this lane's query in each q-block
#pragma unroll
  for (int u = 0; u < QB; ++u) qi[u] = wq_lo + 32 * u + l32;
  const float c = rsqrtf((float)HD) * kLog2e;
  DropSlab ds;
  uint64_t dslab = 0;
  bool dpair = false;
  if constexpr (DROP) {
    dslab = doff + (uint64_t)(b * H + h) * T_ * T_;
    ds.init(seed, dslab);
    dpair = ((doff | (uint64_t)T_) & 1) == 0;
  }

  // ---- Q fragments (B operand): Q[qi][16kk + 8hh + 0..7]
  v8 qf[QB][KK];
#pragma unroll
  for (int u = 0; u < QB; ++u)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      if (qi[u] < T_) qf[u][kk] = *reinterpret_cast<const v8*>(qbase + (long)qi[u] * rs + kk * 16 + hh * 8);
      else qf[u][kk] = v8{};
    }
#pragma unroll
  for (int u = 0; u < QB; ++u)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) asm volatile("" ::"v"(qf[u][kk]));  // retire before the loop

  f32x16 o[QB][DT];
#pragma unroll
  for (int u = 0; u < QB; ++u)
#pragma unroll
    for (int i = 0; i < DT; ++i) o[u][i] = f32x16{};
  float m[QB], l[QB];
#pragma unroll
  for (int u = 0; u < QB; ++u) m[u] = -1e30f, l[u] = 0.f;

  // ---- loop-invariant per-lane offsets
  int koff[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) koff[kk] = k_off<HD>(l32, kk * 2 + hh);
  int voff[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) voff[dt] = v_off<HD>(4 * hh + qrow, dt * 32 + gl * 16 + pcol * 4);
  // DMA piece i of this lane: row P / CH, physical 16-B chunk P % CH (P = (w LD + i) 64 + lane);
  // the source chunk carries the image's XOR swizzle.  Recomputed at every issue from an opaque
  // copy of the lane id (kept in VGPRs across the loop they were spilled at hd 128, and each
  // scratch reload's vmcnt(0) serialised the DMA pieces); the full-tile path below splits P into
  // a wave-uniform row (SGPR base) and the lane's row / chunk with unsigned shifts (23 VALU per
  // 8 pieces instead of 61), this general form serves the sequence-tail tile.
  const uint32_t rs2 = (uint32_t)rs * 2u;  // row stride in bytes (< 2^24 for every shape)
  auto piece = [&](int i, int ln, int& r, int& kc16, int& vc16) {
    const int P = (w * LD + i) * 64 + ln;
    r = P / CH;
    const int pc = P % CH;
    if constexpr (HD == 128) kc16 = pc ^ (r & 15); else kc16 = pc ^ ((r >> 1) & 7);
    const int c64 = (pc >> 2) ^ (HD == 128 ? (r & 3) : ((r >> 1) & 1));
    vc16 = c64 * 4 + (pc & 3);
  };
  const uint32_t smem_u = lds_u32(smem);
  // K / V bases in SGPRs once (the per-piece row offsets are then scalar arithmetic)
  const char* ksb = (const char*)sgpr_ptr(kbase);
  const char* vsb = (const char*)sgpr_ptr(vbase);

  const int kend = causal ? min(T_, q0 + BQ) : T_;
  const int ntiles = (kend + FWD_BK - 1) / FWD_BK;
  const int nact = wq_lo >= T_ ? 0 : (causal ? min(ntiles, min(wq_hi, T_ - 1) / FWD_BK + 1) : ntiles);

  // K/V tiles land in LDS by direct DMA (1 KiB per wave instruction, lane-linear destination);
  // the XOR swizzle is applied to the per-lane SOURCE offset, so the linear DMA image IS the
  // swizzled layout.
  auto issue = [&](int t, int buf) {
    const int k0 = t * FWD_BK;
    const uint32_t base = smem_u + buf * 2 * TILE_B;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    if (k0 + FWD_BK <= T_) {
      // piece i of lane ln: row rb_i + lr (rb_i = (w LD + i) 64 / CH, wave-uniform, folded into the
      // SGPR base), chunk pc = ln % CH; unsigned shifts, and the V chunk does not depend on i
      const uint32_t lr = (uint32_t)ln / CH, pc = (uint32_t)ln % CH;
      const uint32_t lro = lr * rs2;
#pragma unroll
      for (int i = 0; i < LD; ++i) {
        const int rb = (w * LD + i) * (64 / CH);
        const uint32_t r = (uint32_t)rb + lr;
        uint32_t kc16, c64;
        if constexpr (HD == 128) {
          kc16 = pc ^ (r & 15u);
          c64 = (pc >> 2) ^ (r & 3u);
        } else {
          kc16 = pc ^ ((r >> 1) & 7u);
          c64 = (pc >> 2) ^ ((r >> 1) & 1u);
        }
        const uint32_t vc16 = c64 * 4u + (pc & 3u);
        const void* ks = ksb + (long)(k0 + rb) * rs2;
        const void* vs = vsb + (long)(k0 + rb) * rs2;
        const uint32_t pd = (w * LD + i) * 1024;
        glds16s(ks, lro + kc16 * 16u, base + pd);
        glds16s(vs, lro + vc16 * 16u, base + TILE_B + pd);
      }
    } else {  // sequence tail: clamp rows (masked / multiplied by P = 0 later)
      char* kb = smem + buf * 2 * TILE_B;
#pragma unroll
      for (int i = 0; i < LD; ++i) {
        int r, kc16, vc16;
        piece(i, ln, r, kc16, vc16);
        const int pd = (w * LD + i) * 1024;
        const int key = min(k0 + r, T_ - 1);
        glds16(kbase + (long)key * rs + kc16 * 8, kb + pd);
        glds16(vbase + (long)key * rs + vc16 * 8, kb + TILE_B + pd);
      }
    }
  };
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
  int t = 0, buf = 0;
  // dropout keep-mask words of the last computed tile (kmask != nullptr): stored at the top of
  // the next iteration, BEFORE that iteration's DMA issue -- vector memory completes in order,
  // so the ring's counted waits are not lengthened by the stores
  uint32_t kw_pend[QB][NKT];
  int kw_n = 0, kw_t = 0;
  const long kw_row = (long)((T_ + 31) / 32) * T_;  // words per (b, h)
  auto flush_mask = [&]() {
    if constexpr (DROP) {
      if (kmask != nullptr && hh == 0) {
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          if (qi[u] >= T_) continue;
          uint32_t* mrow = kmask + (long)(b * H + h) * kw_row + qi[u];
#pragma unroll
          for (int kt = 0; kt < NKT; ++kt)
            if (kt < kw_n) mrow[(long)(kw_t * NKT + kt) * T_] = kw_pend[u][kt];
        }
      }
      kw_n = 0;
    }
  };
  // One K/V tile.  NV = 32-key sub-tiles this wave can see (< NKT only on causal-diagonal or
  // tail tiles: even waves' diagonal tile has its upper half above every query), EDGE = some
  // visible key is masked.  Instantiated per (NV, EDGE) so each path is straight-line code.
  auto body = [&](auto nv_c, auto edge_c, int k0, const char* kb, const char* vb) {
    constexpr int NV = decltype(nv_c)::value;
    constexpr bool EDGE = decltype(edge_c)::value;
    // ---- S^T = K Q^T for the visible 32-key sub-tiles; each K fragment feeds QB MFMAs
    f32x16 s[QB][NV];
    {
      // the NV sub-tiles' chains interleaved, K fragments of step kk+1 read before the MFMAs of
      // step kk: NV reads in flight under every MFMA pair instead of read -> wait -> MFMA
      v8 cur[NV];
#pragma unroll
      for (int kt = 0; kt < NV; ++kt) {
        cur[kt] = *reinterpret_cast<const v8*>(kb + kt * 32 * ROWB + koff[0]);
#pragma unroll
        for (int u = 0; u < QB; ++u) s[u][kt] = f32x16{};
      }
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        v8 nxt[NV];
        if (kk + 1 < KK) {
#pragma unroll
          for (int kt = 0; kt < NV; ++kt) nxt[kt] = *reinterpret_cast<const v8*>(kb + kt * 32 * ROWB + koff[kk + 1]);
        }
        // keep the next step's reads ahead of this step's MFMAs (the scheduler otherwise sinks
        // them to just before their use and every MFMA pair waits on a fresh LDS read)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kt = 0; kt < NV; ++kt)
#pragma unroll
          for (int u = 0; u < QB; ++u) s[u][kt] = MF<T>::mma(cur[kt], qf[u][kk], s[u][kt]);
        __builtin_amdgcn_sched_barrier(0);
        if (kk + 1 < KK) {
#pragma unroll
          for (int kt = 0; kt < NV; ++kt) cur[kt] = nxt[kt];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      // ---- mask: key k0 + 4hh + off is visible iff off <= lim (one compare + select each)
      if constexpr (EDGE) {
        const int lim = (causal ? min(qi[u], T_ - 1) : T_ - 1) - (k0 + 4 * hh);
#pragma unroll
        for (int kt = 0; kt < NV; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kt * 32 + (r & 3) + 8 * (r >> 2) > lim) s[u][kt][r] = -INFINITY;
      }
      // ---- online softmax
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NV; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[u][kt][r]);
      {  // other half's max: one v_permlane32_swap (no LDS round trip / lgkmcnt wait)
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(mx, fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]))) * c;
      }
      // deferred rescale: only when some lane's max grew by more than kRescaleThr (log2 units);
      // until then P is exponentiated against the stale max and stays below 2^kRescaleThr
      // (fp32 O / l accumulators; bf16 P keeps its relative precision), and the epilogue's
      // lse = m + log2(l) is exact for whatever m the sums were taken against
      if (__builtin_amdgcn_ballot_w64(mx > m[u] + kRescaleThr)) {
        const float mn = fmaxf(m[u], mx);
        const float alpha = __builtin_amdgcn_exp2f(m[u] - mn);
        l[u] *= alpha;
#pragma unroll
        for (int i = 0; i < DT; ++i) o[u][i] *= alpha;
        m[u] = mn;
      }
      float ls = 0.f;
      {  // four partial sums: no 32-deep dependent add chain
        float l4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < NV; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(s[u][kt][r], c, -m[u]));
            l4[r & 3] += pv;
            s[u][kt][r] = pv;
          }
        ls = (l4[0] + l4[1]) + (l4[2] + l4[3]);
      }
      l[u] += ls;
      if constexpr (DROP) {
        // keys (r, r+1) with r even are adjacent: one hash serves both when the row base is even.
        // The keep bits also go to the backward's mask (bit (r&3) + 8(r>>2) + 4hh of the word of
        // this query and 32-key sub-tile; the two lane halves' bits are merged by one swap).
        // Element e0 + o (o = (r&3) + 8(r>>2) <= 27) of this sub-tile row is hashed as pair
        // pb + off: the 64-bit base and both candidate window seeds are formed once per sub-tile,
        // each pair then costs a 32-bit add, a carry select and one mix32 (same values as
        // DropSlab::pair_hash: the low word wraps at most once, into the next window).
        const uint64_t rowbase = dslab + (uint64_t)qi[u] * T_;
#pragma unroll
        for (int kt = 0; kt < NV; ++kt) {
          uint32_t kbits = 0;
          const uint64_t e0 = rowbase + (uint64_t)(k0 + kt * 32 + 4 * hh);
          const uint32_t plo = (uint32_t)(e0 >> 1), phi = (uint32_t)(e0 >> 33);
          const uint32_t smA = phi == ds.hi0 ? ds.sm0 : ds.sm1;
          const uint32_t smB = phi + 1u == ds.hi0 ? ds.sm0 : ds.sm1;
          auto hash_at = [&](uint32_t off) {
            const uint32_t lo = plo + off;
            return mix32(lo ^ (lo < plo ? smB : smA));
          };
          if (dpair) {  // e0 even: keys (r, r+1) share pair pb + o/2
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const uint32_t hv = hash_at((uint32_t)(((r & 3) + 8 * (r >> 2)) >> 1));
              const bool k0b = (hv & 0xFFFFu) >= thr, k1b = (hv >> 16) >= thr;
              s[u][kt][r] = k0b ? s[u][kt][r] * inv_keep : 0.f;
              s[u][kt][r + 1] = k1b ? s[u][kt][r + 1] * inv_keep : 0.f;
              kbits |= ((uint32_t)k0b << ((r & 3) + 8 * (r >> 2))) |
                       ((uint32_t)k1b << (((r + 1) & 3) + 8 * (r >> 2)));
            }
          } else {  // odd T or offset: element e0 + o is half (o+par)&1 of pair pb + (o+par)/2
            const int par = (int)(e0 & 1);
            uint32_t hv[4][3];
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
              for (int j = 0; j < 3; ++j) hv[g][j] = hash_at((uint32_t)(4 * g + j));
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int cr = r & 3;  // compile-time hash indices; par picks between them
              const uint32_t h = par ? hv[r >> 2][(cr + 1) >> 1] : hv[r >> 2][cr >> 1];
              const bool hi = par ? ((cr + 1) & 1) : (cr & 1);
              const bool kb_ = (hi ? (h >> 16) : (h & 0xFFFFu)) >= thr;
              s[u][kt][r] = kb_ ? s[u][kt][r] * inv_keep : 0.f;
              kbits |= (uint32_t)kb_ << ((r & 3) + 8 * (r >> 2));
            }
          }
          if (kmask != nullptr) {
            const uint32_t mine = kbits << (4 * hh);
            const auto sw = __builtin_amdgcn_permlane32_swap(mine, mine, false, false);
            kw_pend[u][kt] = mine | sw[0] | sw[1];
          }
        }
        kw_n = NV;
      }
    }
    // ---- O^T += V^T P^T: P fragments packed from the accumulators, V^T by transposed reads
    //      (each V^T fragment feeds QB MFMAs)
    auto vread = [&](int kt, int s2, int dt) {
      const int off = voff[dt] + (kt * 32 + s2 * 16) * ROWB;
      const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + off));
      const s16x4 r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + off + 8 * ROWB));
      return __builtin_bit_cast(v8, __builtin_shufflevector(r1, r2, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    {
      // one flat sequence of (kt, s2, dt) MFMAs with the next V^T fragment read before each one
      constexpr int NPV = NV * 2 * DT;
      v8 vcur = vread(0, 0, 0);
      v8 pf[QB];
#pragma unroll
      for (int i = 0; i < NPV; ++i) {
        const int kt = i / (2 * DT), s2 = (i / DT) & 1, dt = i % DT;
        v8 vnxt;
        if (i + 1 < NPV) vnxt = vread((i + 1) / (2 * DT), ((i + 1) / DT) & 1, (i + 1) % DT);
        if (dt == 0) {
#pragma unroll
          for (int u = 0; u < QB; ++u) {
            uint32_t uu[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) uu[j] = pack2<T>(s[u][kt][8 * s2 + 2 * j], s[u][kt][8 * s2 + 2 * j + 1]);
            __builtin_memcpy(&pf[u], uu, 16);
          }
        }
#pragma unroll
        for (int u = 0; u < QB; ++u) o[u][dt] = MF<T>::mma(vcur, pf[u], o[u][dt]);
        if (i + 1 < NPV) vcur = vnxt;
      }
    }
  };
  using Ic1 = std::integral_constant<int, 1>;
  using IcN = std::integral_constant<int, NKT>;
  using Yes = std::true_type;
  using No = std::false_type;
  // Interior tiles (no masked key for any of the wave's queries: below the causal diagonal,
  // inside the sequence) form a prefix of the wave's tiles; they run in a loop of their own with
  // the one unmasked body, so the O accumulators never meet the edge variants' registers on the
  // hot path (a shared loop made hipcc copy them between variants every tile).
  const int n_int = wq_hi >= T_ ? 0 : min(min(nact, T_ / FWD_BK), causal ? (wq_lo + 1) / FWD_BK : nact);
  for (; t < n_int; ++t) {
    flush_mask();  // keep bits of tile t - 1
    if (t + NBUF - 1 < ntiles) issue(t + NBUF - 1, buf == 0 ? NBUF - 1 : buf - 1);
    kw_t = t;
    const char* kb = smem + buf * 2 * TILE_B;
    body(IcN{}, No{}, t * FWD_BK, kb, kb + TILE_B);
    ring_wait(t);  // the DMA of tile t+1 has landed (asm-issued, so drained by hand)
    buf = buf == NBUF - 1 ? 0 : buf + 1;
  }
  // causal diagonal / sequence tail tiles
  for (; t < nact; ++t) {
    flush_mask();
    if (t + NBUF - 1 < ntiles) issue(t + NBUF - 1, buf == 0 ? NBUF - 1 : buf - 1);
    const int k0 = t * FWD_BK;
    kw_t = t;
    const char* kb = smem + buf * 2 * TILE_B;
    const int kvis = min(causal ? wq_hi : T_ - 1, T_ - 1) - k0;  // >= 0 for an active tile
    if (NKT == 1 || kvis >= 32) body(IcN{}, Yes{}, k0, kb, kb + TILE_B);
    else body(Ic1{}, Yes{}, k0, kb, kb + TILE_B);
    ring_wait(t);
    buf = buf == NBUF - 1 ? 0 : buf + 1;
  }
  flush_mask();
  for (; t < ntiles; ++t) {  // wave done (causal): keep the DMA ring and barriers going
    if (t + NBUF - 1 < ntiles) issue(t + NBUF - 1, buf == 0 ? NBUF - 1 : buf - 1);
    ring_wait(t);
    buf = buf == NBUF - 1 ? 0 : buf + 1;
  }

  // ---- epilogue: combine the two halves' partial sums, normalise, store O and LSE
#pragma unroll
  for (int u = 0; u < QB; ++u) {
    const float lt = l[u] + __shfl_xor(l[u], 32, 64);
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    T* orow = out + ((long)b * T_ + min(qi[u], T_ - 1)) * (long)H * HD + (long)h * HD;
    // 16-B stores: lane (q, half hh) holds d = 8 gq + 4 hh + 0..3 of each 32-column tile; one
    // v_permlane32_swap per dword of a (gq, gq+1) pair leaves 8 contiguous d of group gq in the
    // lower half and of gq+1 in the upper half (cdna_hip_programming.md T21: half the store
    // instructions of the dwordx2 form, same bytes).  Every lane swaps (cross-lane); only the
    // store is guarded.
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; gq += 2) {
        uint32_t ax = pack2<T>(o[u][dt][4 * gq + 0] * inv, o[u][dt][4 * gq + 1] * inv);
        uint32_t ay = pack2<T>(o[u][dt][4 * gq + 2] * inv, o[u][dt][4 * gq + 3] * inv);
        uint32_t bx = pack2<T>(o[u][dt][4 * gq + 4] * inv, o[u][dt][4 * gq + 5] * inv);
        uint32_t by = pack2<T>(o[u][dt][4 * gq + 6] * inv, o[u][dt][4 * gq + 7] * inv);
        const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
        const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
        ax = rx[0]; bx = rx[1]; ay = ry[0]; by = ry[1];
        if (qi[u] < T_)
          *reinterpret_cast<uint4*>(orow + dt * 32 + 8 * gq + 8 * hh) = uint4{ax, ay, bx, by};
      }
    if (qi[u] < T_ && hh == 0) lse[((long)b * H + h) * T_ + qi[u]] = m[u] + log2f(lt);
  }
}

// ---- 8-wave ping-pong forward ----------------------------------------------------------------
// Workgroup = 8 waves, two per SIMD (waves w and w + 4 share one), 256 queries: wave w owns the
// 32-query block 2 (w & 3) + (w >> 2), so both halves carry the same causal load.  Per K/V tile j
// every wave runs two phases separated by s_barrier:
//   cluster(j): O^T += V_{j-1}^T P_{j-1}^T and S_j^T = K_j Q^T -- 32 MFMAs (hd 128) back to back,
//               LDS fragments read one MFMA ahead;
//   softmax(j): mask, online max / deferred rescale, exp2, row sum, P_j packed to bf16 -- VALU.
// Half B (waves 4-7) runs one phase behind half A, so on every SIMD one wave's MFMA chain issues
// while its partner's softmax runs (MI355X_MICROARCH.md "Two waves per SIMD"):
//   phase 2j:   A cluster(j)   B softmax(j-1)
//   phase 2j+1: A softmax(j)   B cluster(j)
// Every wave passes the same 2 (N + 1) barriers (N = the workgroup's tile count); a wave whose
// queries need fewer tiles skips the work, never a barrier.  The rescale of O in softmax(j) comes
// after cluster(j) has added P_{j-1} V_{j-1} (taken against the old max): the safe order of
// cdna_hip_programming.md T13.  K and V rings of two slots each: K_{j+1} and V_j are issued at the
// top of phase 2j (their slots' previous tiles were last read in phase 2j-1) and waited for at
// the end of phase 2j+1, before cluster(j+1) reads them.
template <typename T, int HD, bool DROP>
__global__ __launch_bounds__(512, 1) void attn_fwd_pp_k(const T* __restrict__ qkv, T* __restrict__ out,
                                                       float* __restrict__ lse, int T_, int H, int G, int B_,
                                                       bool causal, uint32_t thr, float inv_keep, uint64_t seed,
                                                       uint64_t doff, uint32_t* __restrict__ kmask,
                                                       unsigned long long* __restrict__ dbg) {
  typedef typename MF<T>::v8 v8;
  constexpr int KK = HD / 16;            // k-steps of QK^T
  constexpr int DT = HD / 32;            // 32-row tiles of O^T
  constexpr int CH = HD / 8;             // 16-B chunks per row
  constexpr int ROWB = HD * 2;
  constexpr int BK = 64;                 // keys per tile
  constexpr int TILE_B = BK * ROWB;      // bytes of one K (or V) tile
  constexpr int PPW = BK * CH / 512;     // 1-KiB DMA pieces per wave per K (or V) tile
  constexpr int BQ = 256;
  constexpr int NPV = 2 * 2 * DT;        // PV MFMAs per tile
  constexpr int NQK = 2 * KK;            // QK MFMAs per tile
  static_assert(PPW >= 1, "tile too small for 8 waves");

  extern __shared__ __attribute__((aligned(16))) char smem[];  // K slots 0-2, V slots 0-2

  const int nqb = (T_ + BQ - 1) / BQ;
  const int lin = blockIdx.x, nbh = H * B_;
  const int qbi = lin / nbh, bh = lin - qbi * nbh;
  const int qb = causal ? nqb - 1 - qbi : qbi;
  const int h = bh % H, b = bh / H;
  const int g = h / (H / G);
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = w >> 2;
  // debug timing (dbg != nullptr, first 16 workgroups): s_memtime before / after every barrier
  int nst = 0;
  auto stamp = [&]() __attribute__((always_inline)) {
    if (dbg != nullptr && blockIdx.x < 16 && lane == 0 && nst < 64)
      dbg[((long)blockIdx.x * 8 + w) * 64 + nst] = __builtin_amdgcn_s_memtime();
    ++nst;
  };
  stamp();
  const int gi = lane & 15, gl = (lane >> 4) & 1, qrow = gi >> 2, pcol = gi & 3;
  const long rs = (long)(H + 2 * G) * HD;
  const T* qbase = qkv + (long)b * T_ * rs + (long)h * HD;
  const T* kbase = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const T* vbase = qkv + (long)b * T_ * rs + (long)(H + G + g) * HD;
  const int q0 = qb * BQ;
  const int wq_lo = q0 + 32 * (2 * (w & 3) + half), wq_hi = wq_lo + 31;
  const int qi = wq_lo + l32;
  const float c = rsqrtf((float)HD) * kLog2e;
  DropSlab ds;
  uint64_t dslab = 0;
  bool dpair = false;
  if constexpr (DROP) {
    dslab = doff + (uint64_t)(b * H + h) * T_ * T_;
    ds.init(seed, dslab);
    dpair = ((doff | (uint64_t)T_) & 1) == 0;
  }

  v8 qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    if (qi < T_) qf[kk] = *reinterpret_cast<const v8*>(qbase + (long)qi * rs + kk * 16 + hh * 8);
    else qf[kk] = v8{};
  }
  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x16{};
  f32x16 s[2];
  v8 pk[2][2];  // P_j packed: [32-key sub-tile][16-key half]; zero = a PV step that adds nothing
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) pk[kt][0] = pk[kt][1] = v8{};
  float m = -1e30f, l = 0.f;

  int koff[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) koff[kk] = k_off<HD>(l32, kk * 2 + hh);
  int voff[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) voff[dt] = v_off<HD>(4 * hh + qrow, dt * 32 + gl * 16 + pcol * 4);

  const uint32_t rs2 = (uint32_t)rs * 2u;
  const uint32_t smem_u = lds_u32(smem);
  const char* ksb = (const char*)sgpr_ptr(kbase);
  const char* vsb = (const char*)sgpr_ptr(vbase);

  const int kend = causal ? min(T_, q0 + BQ) : T_;
  const int N = (kend + BK - 1) / BK;
  const int nact = wq_lo >= T_ ? 0 : (causal ? min(N, min(wq_hi, T_ - 1) / BK + 1) : N);
  const int n_int = wq_hi >= T_ ? 0 : min(min(nact, T_ / BK), causal ? (wq_lo + 1) / BK : nact);

  // DMA of one K (kv = 0) or V (kv = 1) tile: this wave's PPW pieces, lane-linear destination,
  // swizzle applied to the source chunk (the linear image IS the swizzled layout)
  auto issue = [&](int t, int kv) __attribute__((always_inline)) {
    const int k0 = t * BK;
    const uint32_t base = smem_u + (kv * 3 + t % 3) * TILE_B;
    const char* sb = kv ? vsb : ksb;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const uint32_t lr = (uint32_t)ln / CH, pc = (uint32_t)ln % CH;
    const bool full = k0 + BK <= T_;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int rb = (w * PPW + i) * (64 / CH);
      const uint32_t r = (uint32_t)rb + lr;
      uint32_t cc;
      if (kv == 0) {
        cc = HD == 128 ? (pc ^ (r & 15u)) : (pc ^ ((r >> 1) & 7u));
      } else {
        const uint32_t c64 = HD == 128 ? ((pc >> 2) ^ (r & 3u)) : ((pc >> 2) ^ ((r >> 1) & 1u));
        cc = c64 * 4u + (pc & 3u);
      }
      const uint32_t pd = base + (w * PPW + i) * 1024;
      if (full) {
        glds16s(sb + (long)(k0 + rb) * rs2, lr * rs2 + cc * 16u, pd);
      } else {  // sequence tail: rows clamped (masked / multiplied by P = 0 later)
        const int key = min(k0 + rb + (int)lr, T_ - 1);
        glds16((const char*)(kv ? vbase : kbase) + (long)key * rs2 + cc * 16u, smem + (pd - smem_u));
      }
    }
  };

  auto kread = [&](int t, int kt, int kk) __attribute__((always_inline)) {
    const char* kb = smem + (t % 3) * TILE_B;
    return *reinterpret_cast<const v8*>(kb + kt * 32 * ROWB + koff[kk]);
  };
  auto vread = [&](int t, int kt, int s2, int dt) __attribute__((always_inline)) {
    const char* vb = smem + (3 + t % 3) * TILE_B;
    const int off = voff[dt] + (kt * 32 + s2 * 16) * ROWB;
    const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + off));
    const s16x4 r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + off + 8 * ROWB));
    return __builtin_bit_cast(v8, __builtin_shufflevector(r1, r2, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  // Register discipline (hipcc otherwise copies the accumulators at every join of the two
  // phase bodies): O and S are written only by the matrix phase, P / m / l only by the VALU
  // phase.  So the causal / tail mask is applied to S right after the QK MFMAs, and a rescale
  // decided by softmax(j) is applied to O by cluster(j+1), before it adds P_j V_j.
  bool resc = false;
  float ralpha = 1.f;

  // matrix phase: [rescale O] PV of tile j-1 (if pv), then QK of tile j (if qk) [+ mask]: one
  // flat MFMA sequence with the fragment reads RD steps ahead (the partner wave is in its VALU
  // phase, so nothing else fills the matrix pipe while an MFMA waits on its LDS read)
  constexpr int RD = 3;
  auto run = [&](auto i0_c, auto i1_c, int j) __attribute__((always_inline)) {
    constexpr int I0 = decltype(i0_c)::value, I1 = decltype(i1_c)::value;
    auto frag = [&](int i) __attribute__((always_inline)) {
      if (i < NPV) return vread(j - 1, i / (2 * DT), (i / DT) & 1, i % DT);
      const int q = i - NPV;
      return kread(j, q & 1, q >> 1);
    };
    v8 f[NPV + NQK];
#pragma unroll
    for (int i = I0; i < I1 && i < I0 + RD; ++i) f[i] = frag(i);
#pragma unroll
    for (int i = I0; i < I1; ++i) {
      if (i + RD < I1) f[i + RD] = frag(i + RD);
      __builtin_amdgcn_sched_barrier(0);
      if (i < NPV) {
        const int kt = i / (2 * DT), s2 = (i / DT) & 1, dt = i % DT;
        o[dt] = MF<T>::mma(f[i], pk[kt][s2], o[dt]);
      } else {
        const int q = i - NPV;
        s[q & 1] = MF<T>::mma(f[i], qf[q >> 1], s[q & 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using IcZ = std::integral_constant<int, 0>;
  using IcP = std::integral_constant<int, NPV>;
  using IcE = std::integral_constant<int, NPV + NQK>;
  // cluster(j) inside the loop is always the full sequence: a wave past its last tile (causal
  // diagonal) multiplies the zero P written by its null softmax, and its QK result is unused
  auto cluster = [&](auto i0_c, auto i1_c, int j) __attribute__((always_inline)) {
    constexpr int I0 = decltype(i0_c)::value, I1 = decltype(i1_c)::value;
    if (I0 == 0 && resc) {
#pragma unroll
      for (int i = 0; i < DT; ++i) o[i] *= ralpha;
      resc = false;
    }
    if (I1 > NPV) {
      s[0] = f32x16{};
      s[1] = f32x16{};
    }
    run(i0_c, i1_c, j);
    if (I1 > NPV && j >= n_int) {  // key k0 + 4hh + off visible iff off <= lim
      const int lim = (causal ? min(qi, T_ - 1) : T_ - 1) - (j * BK + 4 * hh);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kt * 32 + (r & 3) + 8 * (r >> 2) > lim) s[kt][r] = -INFINITY;
    }
  };

  // VALU phase: online softmax of S_j -> P_j (reads S, writes P, m, l and the pending rescale)
  auto softmax = [&](int j) __attribute__((always_inline)) {
    const int k0 = j * BK;
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kt][r]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(mx, fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]))) * c;
    }
    if (__builtin_amdgcn_ballot_w64(mx > m + kRescaleThr)) {
      const float mn = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      l *= alpha;
      ralpha = resc ? ralpha * alpha : alpha;
      resc = true;
      m = mn;
    }
    float pr[2][16];
    float l4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        pr[kt][r] = __builtin_amdgcn_exp2f(fmaf(s[kt][r], c, -m));
        l4[r & 3] += pr[kt][r];
      }
    l += (l4[0] + l4[1]) + (l4[2] + l4[3]);
    if constexpr (DROP) {
      // same keep bits as attn_fwd_mfma_k (pair hash of adjacent keys when the row base is even)
      const uint64_t rowbase = dslab + (uint64_t)qi * T_;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        uint32_t kbits = 0;
        const uint64_t e0 = rowbase + (uint64_t)(k0 + kt * 32 + 4 * hh);
        const uint32_t plo = (uint32_t)(e0 >> 1), phi = (uint32_t)(e0 >> 33);
        const uint32_t smA = phi == ds.hi0 ? ds.sm0 : ds.sm1;
        const uint32_t smB = phi + 1u == ds.hi0 ? ds.sm0 : ds.sm1;
        auto hash_at = [&](uint32_t off) __attribute__((always_inline)) {
          const uint32_t lo = plo + off;
          return mix32(lo ^ (lo < plo ? smB : smA));
        };
        if (dpair) {
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const uint32_t hv = hash_at((uint32_t)(((r & 3) + 8 * (r >> 2)) >> 1));
            const bool k0b = (hv & 0xFFFFu) >= thr, k1b = (hv >> 16) >= thr;
            pr[kt][r] = k0b ? pr[kt][r] * inv_keep : 0.f;
            pr[kt][r + 1] = k1b ? pr[kt][r + 1] * inv_keep : 0.f;
            kbits |= ((uint32_t)k0b << ((r & 3) + 8 * (r >> 2))) | ((uint32_t)k1b << (((r + 1) & 3) + 8 * (r >> 2)));
          }
        } else {
          const int par = (int)(e0 & 1);
          uint32_t hv[4][3];
#pragma unroll
          for (int gg = 0; gg < 4; ++gg)
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) hv[gg][jj] = hash_at((uint32_t)(4 * gg + jj));
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int cr = r & 3;
            const uint32_t hx = par ? hv[r >> 2][(cr + 1) >> 1] : hv[r >> 2][cr >> 1];
            const bool hi = par ? ((cr + 1) & 1) : (cr & 1);
            const bool kb_ = (hi ? (hx >> 16) : (hx & 0xFFFFu)) >= thr;
            pr[kt][r] = kb_ ? pr[kt][r] * inv_keep : 0.f;
            kbits |= (uint32_t)kb_ << ((r & 3) + 8 * (r >> 2));
          }
        }
        if (kmask != nullptr) {
          const uint32_t mine = kbits << (4 * hh);
          const auto sw = __builtin_amdgcn_permlane32_swap(mine, mine, false, false);
          const int kw = j * 2 + kt, nkw = (T_ + 31) / 32;  // the tail tile's second word may not exist
          if (hh == 0 && qi < T_ && kw < nkw)
            kmask[(long)(b * H + h) * ((long)nkw * T_) + (long)kw * T_ + qi] = mine | sw[0] | sw[1];
        }
      }
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        uint32_t uu[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) uu[jj] = pack2<T>(pr[kt][8 * s2 + 2 * jj], pr[kt][8 * s2 + 2 * jj + 1]);
        __builtin_memcpy(&pk[kt][s2], uu, 16);
      }
  };

  // VALU phase body: the real softmax for a tile this wave needs, else P = 0
  auto vphase = [&](int j) __attribute__((always_inline)) {
    if (j < nact) {
      softmax(j);
    } else {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) pk[kt][0] = pk[kt][1] = v8{};
    }
  };

  // DMA step s (issued by every wave at the end of its VALU phase of pair s): K_{s+2}, V_{s+1}.
  // K_t's slot was last read in phase 2t-5, V_t's in 2t-3: both before the step's phases.  The
  // wait at the end of phase 2s+1 needs step s-1's pieces (K_{s+1}, V_s) only: the counted vmcnt
  // leaves step s's pieces in flight.
  auto dma_step = [&](int st) __attribute__((always_inline)) {
    if (st + 2 < N) issue(st + 2, 0);
    if (st + 1 < N) issue(st + 1, 1);
  };
  auto dma_wait = [&](int st) __attribute__((always_inline)) {
    if (st + 2 < N) wait_vm<2 * PPW>();
    else if (st + 1 < N) wait_vm<PPW>();
    else wait_vm0();
  };

  if (N > 0) issue(0, 0);
  if (N > 1) issue(1, 0);
  if (N > 0) issue(0, 1);
  wait_vm0();
  stamp();
  __builtin_amdgcn_s_barrier();
  stamp();
  if (N > 0) {
    // phases 0, 1 (tile 0: QK only)
    if (half == 0) cluster(IcP{}, IcE{}, 0); else dma_step(0);
    asm volatile("" ::: "memory");
    stamp();
    __builtin_amdgcn_s_barrier();
    stamp();
    if (half == 0) {
      vphase(0);
      dma_step(0);
    } else {
      cluster(IcP{}, IcE{}, 0);
    }
    dma_wait(0);
    stamp();
    __builtin_amdgcn_s_barrier();
    stamp();
    // phases 2 .. 2N-1: half A runs cluster(p / 2) on even p and the VALU phase of (p - 1) / 2 on
    // odd p, half B one phase later; one instance of each body.  DMA step p / 2 follows the VALU
    // phase of either half.
    for (int p = 2; p < 2 * N; ++p) {
      if (((p + half) & 1) == 0) {
        cluster(IcZ{}, IcE{}, (p - half) >> 1);
      } else if constexpr (DROP) {  // keep-mask stores before the step's pieces (counted waits)
        vphase((p - 1 - half) >> 1);
        dma_step(p >> 1);
      } else {  // the pieces' issue overlaps the softmax's dependency stalls
        dma_step(p >> 1);
        vphase((p - 1 - half) >> 1);
      }
      if (p & 1) dma_wait(p >> 1);
      else asm volatile("" ::: "memory");
      stamp();
      __builtin_amdgcn_s_barrier();
      stamp();
    }
    // phases 2N, 2N+1 (PV of the last tile)
    if (half == 0) cluster(IcZ{}, IcP{}, N); else vphase(N - 1);
    asm volatile("" ::: "memory");
    stamp();
    __builtin_amdgcn_s_barrier();
    stamp();
    if (half != 0) cluster(IcZ{}, IcP{}, N);
  }

  // ---- epilogue (as attn_fwd_mfma_k)
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  T* orow = out + ((long)b * T_ + min(qi, T_ - 1)) * (long)H * HD + (long)h * HD;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int gq = 0; gq < 4; gq += 2) {
      uint32_t ax = pack2<T>(o[dt][4 * gq + 0] * inv, o[dt][4 * gq + 1] * inv);
      uint32_t ay = pack2<T>(o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv);
      uint32_t bx = pack2<T>(o[dt][4 * gq + 4] * inv, o[dt][4 * gq + 5] * inv);
      uint32_t by = pack2<T>(o[dt][4 * gq + 6] * inv, o[dt][4 * gq + 7] * inv);
      const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
      ax = rx[0]; bx = rx[1]; ay = ry[0]; by = ry[1];
      if (qi < T_) *reinterpret_cast<uint4*>(orow + dt * 32 + 8 * gq + 8 * hh) = uint4{ax, ay, bx, by};
    }
  if (qi < T_ && hh == 0) lse[((long)b * H + h) * T_ + qi] = m + log2f(lt);
}

// ---- software-pipelined forward ----------------------------------------------------------------
// Same workgroup shape as attn_fwd_mfma_k (4 waves x 32 queries, 2 workgroups per CU), but each
// wave overlaps its own VALU work with its MFMA chain (FA3-style intra-wave pipelining; the
// partner wave of the SIMD belongs to the other workgroup and is not synchronised with it):
//   iteration t:  S_t = K_t Q^T      (16 MFMAs at hd 128)  ||  exp / sum / pack of S_{t-1} -> P_{t-1}
//                 O += V_{t-1} P_{t-1}  (16 MFMAs)          ||  row max of S_t, rescale decision
// The VALU half of the softmax of tile t-1 fills the MFMA issue gaps of tile t instead of running
// between two MFMA chains (MI355X_MICROARCH.md: up to ~5 single-issue instructions hide per
// 32x32x16 MFMA gap).  K and V rings of two slots each: K_{t+1} and V_t are issued at the top of
// iteration t (K_{t-1} and V_{t-2}, their slots' previous tiles, were read in iteration t-1).
// S is double-buffered by unrolling the interior loop by two (named buffers, no copies).
template <typename T, int HD, bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd_sp_k(const T* __restrict__ qkv, T* __restrict__ out,
                                                       float* __restrict__ lse, int T_, int H, int G, int B_,
                                                       bool causal, uint32_t thr, float inv_keep, uint64_t seed,
                                                       uint64_t doff, uint32_t* __restrict__ kmask) {
  typedef typename MF<T>::v8 v8;
  constexpr int KK = HD / 16;
  constexpr int DT = HD / 32;
  constexpr int CH = HD / 8;
  constexpr int ROWB = HD * 2;
  constexpr int BK = 64;
  constexpr int TILE_B = BK * ROWB;
  constexpr int PPW = BK * CH / 256;     // 1-KiB DMA pieces per wave per K (or V) tile
  constexpr int BQ = 128;
  constexpr int NPV = 2 * 2 * DT;
  constexpr int NQK = 2 * KK;

  extern __shared__ __attribute__((aligned(16))) char smem[];  // K slots 0, 1, V slots 0, 1

  const int nqb = (T_ + BQ - 1) / BQ;
  const int lin = blockIdx.x, nbh = H * B_;
  const int qbi = lin / nbh, bh = lin - qbi * nbh;
  const int qb = causal ? nqb - 1 - qbi : qbi;
  const int h = bh % H, b = bh / H;
  const int g = h / (H / G);
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gi = lane & 15, gl = (lane >> 4) & 1, qrow = gi >> 2, pcol = gi & 3;
  const long rs = (long)(H + 2 * G) * HD;
  const T* qbase = qkv + (long)b * T_ * rs + (long)h * HD;
  const T* kbase = qkv + (long)b * T_ * rs + (long)(H + g) * HD;
  const T* vbase = qkv + (long)b * T_ * rs + (long)(H + G + g) * HD;
  const int q0 = qb * BQ;
  const int wq_lo = q0 + 32 * w, wq_hi = wq_lo + 31;
  const int qi = wq_lo + l32;
  const float c = rsqrtf((float)HD) * kLog2e;
  DropSlab ds;
  uint64_t dslab = 0;
  bool dpair = false;
  if constexpr (DROP) {
    dslab = doff + (uint64_t)(b * H + h) * T_ * T_;
    ds.init(seed, dslab);
    dpair = ((doff | (uint64_t)T_) & 1) == 0;
  }

  v8 qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    if (qi < T_) qf[kk] = *reinterpret_cast<const v8*>(qbase + (long)qi * rs + kk * 16 + hh * 8);
    else qf[kk] = v8{};
  }
  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x16{};
  f32x16 sa[2], sb[2];
  v8 pk[2][2];
  float m = -1e30f, l = 0.f;

  int koff[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) koff[kk] = k_off<HD>(l32, kk * 2 + hh);
  int voff[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) voff[dt] = v_off<HD>(4 * hh + qrow, dt * 32 + gl * 16 + pcol * 4);

  const uint32_t rs2 = (uint32_t)rs * 2u;
  const uint32_t smem_u = lds_u32(smem);
  const char* ksb = (const char*)sgpr_ptr(kbase);
  const char* vsb = (const char*)sgpr_ptr(vbase);

  const int kend = causal ? min(T_, q0 + BQ) : T_;
  const int N = (kend + BK - 1) / BK;
  const int nact = wq_lo >= T_ ? 0 : (causal ? min(N, min(wq_hi, T_ - 1) / BK + 1) : N);
  const int n_int = wq_hi >= T_ ? 0 : min(min(nact, T_ / BK), causal ? (wq_lo + 1) / BK : nact);

  auto issue = [&](int t, int kv) __attribute__((always_inline)) {
    const int k0 = t * BK;
    const uint32_t base = smem_u + (kv * 2 + (t & 1)) * TILE_B;
    const char* sbase = kv ? vsb : ksb;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const uint32_t lr = (uint32_t)ln / CH, pc = (uint32_t)ln % CH;
    if (k0 + BK <= T_) {
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        const int rb = (w * PPW + i) * (64 / CH);
        const uint32_t r = (uint32_t)rb + lr;
        uint32_t cc;
        if (kv == 0) {
          cc = HD == 128 ? (pc ^ (r & 15u)) : (pc ^ ((r >> 1) & 7u));
        } else {
          const uint32_t c64 = HD == 128 ? ((pc >> 2) ^ (r & 3u)) : ((pc >> 2) ^ ((r >> 1) & 1u));
          cc = c64 * 4u + (pc & 3u);
        }
        glds16s(sbase + (long)(k0 + rb) * rs2, lr * rs2 + cc * 16u, base + (w * PPW + i) * 1024);
      }
    } else {  // sequence tail: rows clamped (masked / multiplied by P = 0 later)
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        const int rb = (w * PPW + i) * (64 / CH);
        const uint32_t r = (uint32_t)rb + lr;
        uint32_t cc;
        if (kv == 0) {
          cc = HD == 128 ? (pc ^ (r & 15u)) : (pc ^ ((r >> 1) & 7u));
        } else {
          const uint32_t c64 = HD == 128 ? ((pc >> 2) ^ (r & 3u)) : ((pc >> 2) ^ ((r >> 1) & 1u));
          cc = c64 * 4u + (pc & 3u);
        }
        const int key = min(k0 + (int)r, T_ - 1);
        glds16((const char*)(kv ? vbase : kbase) + (long)key * rs2 + cc * 16u,
               smem + (kv * 2 + (t & 1)) * TILE_B + (w * PPW + i) * 1024);
      }
    }
  };
  auto kread = [&](int t, int kt, int kk) __attribute__((always_inline)) {
    return *reinterpret_cast<const v8*>(smem + (t & 1) * TILE_B + kt * 32 * ROWB + koff[kk]);
  };
  auto vread = [&](int t, int kt, int s2, int dt) __attribute__((always_inline)) {
    const char* vb = smem + (2 + (t & 1)) * TILE_B;
    const int off = voff[dt] + (kt * 32 + s2 * 16) * ROWB;
    const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + off));
    const s16x4 r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + off + 8 * ROWB));
    return __builtin_bit_cast(v8, __builtin_shufflevector(r1, r2, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  // S_t = K_t Q^T into s_out (K fragments one step ahead)
  auto qk = [&](f32x16 (&so)[2], int t) __attribute__((always_inline)) {
    so[0] = f32x16{};
    so[1] = f32x16{};
    v8 c0 = kread(t, 0, 0), c1 = kread(t, 1, 0);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      v8 n0, n1;
      if (kk + 1 < KK) {
        n0 = kread(t, 0, kk + 1);
        n1 = kread(t, 1, kk + 1);
      }
      so[0] = MF<T>::mma(c0, qf[kk], so[0]);
      so[1] = MF<T>::mma(c1, qf[kk], so[1]);
      if (kk + 1 < KK) {
        c0 = n0;
        c1 = n1;
      }
    }
  };
  auto mask = [&](f32x16 (&so)[2], int t) __attribute__((always_inline)) {
    const int lim = (causal ? min(qi, T_ - 1) : T_ - 1) - (t * BK + 4 * hh);
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kt * 32 + (r & 3) + 8 * (r >> 2) > lim) so[kt][r] = -INFINITY;
  };
  // row max of S_t and the (deferred) rescale decision; the O rescale itself runs after the
  // PV of tile t-1 (taken against the old max), i.e. right here at the end of the iteration
  auto decide = [&](const f32x16 (&si)[2]) __attribute__((always_inline)) {
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, si[kt][r]);
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
    mx = fmaxf(mx, fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]))) * c;
    if (__builtin_amdgcn_ballot_w64(mx > m + kRescaleThr)) {
      const float mn = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      l *= alpha;
#pragma unroll
      for (int i = 0; i < DT; ++i) o[i] *= alpha;
      m = mn;
    }
  };
  // dropout of sub-tile kt of P_{t-1} (pr = its exp values) and its keep-mask word
  auto dropout = [&](float (&pr)[16], int kt, int t) __attribute__((always_inline)) {
    if constexpr (DROP) {
      const uint64_t rowbase = dslab + (uint64_t)qi * T_;
      uint32_t kbits = 0;
      const uint64_t e0 = rowbase + (uint64_t)(t * BK + kt * 32 + 4 * hh);
      const uint32_t plo = (uint32_t)(e0 >> 1), phi = (uint32_t)(e0 >> 33);
      const uint32_t smA = phi == ds.hi0 ? ds.sm0 : ds.sm1;
      const uint32_t smB = phi + 1u == ds.hi0 ? ds.sm0 : ds.sm1;
      auto hash_at = [&](uint32_t off) __attribute__((always_inline)) {
        const uint32_t lo = plo + off;
        return mix32(lo ^ (lo < plo ? smB : smA));
      };
      if (dpair) {
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const uint32_t hv = hash_at((uint32_t)(((r & 3) + 8 * (r >> 2)) >> 1));
          const bool k0b = (hv & 0xFFFFu) >= thr, k1b = (hv >> 16) >= thr;
          pr[r] = k0b ? pr[r] * inv_keep : 0.f;
          pr[r + 1] = k1b ? pr[r + 1] * inv_keep : 0.f;
          kbits |= ((uint32_t)k0b << ((r & 3) + 8 * (r >> 2))) | ((uint32_t)k1b << (((r + 1) & 3) + 8 * (r >> 2)));
        }
      } else {
        const int par = (int)(e0 & 1);
        uint32_t hv[4][3];
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
#pragma unroll
          for (int jj = 0; jj < 3; ++jj) hv[gg][jj] = hash_at((uint32_t)(4 * gg + jj));
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int cr = r & 3;
          const uint32_t hx = par ? hv[r >> 2][(cr + 1) >> 1] : hv[r >> 2][cr >> 1];
          const bool hi = par ? ((cr + 1) & 1) : (cr & 1);
          const bool kb_ = (hi ? (hx >> 16) : (hx & 0xFFFFu)) >= thr;
          pr[r] = kb_ ? pr[r] * inv_keep : 0.f;
          kbits |= (uint32_t)kb_ << ((r & 3) + 8 * (r >> 2));
        }
      }
      if (kmask != nullptr) {
        const uint32_t mine = kbits << (4 * hh);
        const auto sw = __builtin_amdgcn_permlane32_swap(mine, mine, false, false);
        const int kw = t * 2 + kt, nkw = (T_ + 31) / 32;
        if (hh == 0 && qi < T_ && kw < nkw)
          kmask[(long)(b * H + h) * ((long)nkw * T_) + (long)kw * T_ + qi] = mine | sw[0] | sw[1];
      }
    }
  };
  auto pack = [&](const float (&pr)[16], int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      uint32_t uu[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) uu[jj] = pack2<T>(pr[8 * s2 + 2 * jj], pr[8 * s2 + 2 * jj + 1]);
      __builtin_memcpy(&pk[kt][s2], uu, 16);
    }
  };
  // steady-state iteration t (1 <= t < nact): S_t = K_t Q^T into so with the softmax of sub-tile 0
  // of si (= S_{t-1}) in the MFMA gaps, then O += V_{t-1} P_{t-1} with sub-tile 1's softmax in the
  // first half's gaps and the row max of S_t in the second half's; source order = issue order
  // (sched_barrier pins every group)
  constexpr int E0 = 16 / KK;            // sub-tile-0 elements per QK k-step
  constexpr int E1 = 16 / (NPV / 2);     // sub-tile-1 elements per PV MFMA (first half)
  constexpr int EM = 32 / (NPV / 2);     // S_t elements maxed per PV MFMA (second half)
  auto steady = [&](f32x16 (&si)[2], f32x16 (&so)[2], int t, bool edge) __attribute__((always_inline)) {
    float pr0[16], pr1[16];
    float l4[4] = {0.f, 0.f, 0.f, 0.f};
    so[0] = f32x16{};
    so[1] = f32x16{};
    {
      v8 c0 = kread(t, 0, 0), c1 = kread(t, 1, 0);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        v8 n0, n1;
        if (kk + 1 < KK) {
          n0 = kread(t, 0, kk + 1);
          n1 = kread(t, 1, kk + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        so[0] = MF<T>::mma(c0, qf[kk], so[0]);
#pragma unroll
        for (int e = 0; e < E0 / 2; ++e) {
          const int r = kk * E0 + e;
          pr0[r] = __builtin_amdgcn_exp2f(fmaf(si[0][r], c, -m));
          l4[r & 3] += pr0[r];
        }
        so[1] = MF<T>::mma(c1, qf[kk], so[1]);
#pragma unroll
        for (int e = E0 / 2; e < E0; ++e) {
          const int r = kk * E0 + e;
          pr0[r] = __builtin_amdgcn_exp2f(fmaf(si[0][r], c, -m));
          l4[r & 3] += pr0[r];
        }
        __builtin_amdgcn_sched_barrier(0);
        if (kk + 1 < KK) {
          c0 = n0;
          c1 = n1;
        }
      }
    }
    dropout(pr0, 0, t - 1);
    pack(pr0, 0);
    if (edge) mask(so, t);
    float mx = -INFINITY;
    {
      v8 cur = vread(t - 1, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < NPV; ++i) {
        const int kt = i / (2 * DT), s2 = (i / DT) & 1, dt = i % DT;
        v8 nxt;
        if (i + 1 < NPV) nxt = vread(t - 1, (i + 1) / (2 * DT), ((i + 1) / DT) & 1, (i + 1) % DT);
        __builtin_amdgcn_sched_barrier(0);
        o[dt] = MF<T>::mma(cur, pk[kt][s2], o[dt]);
        if (i < NPV / 2) {
#pragma unroll
          for (int e = 0; e < E1; ++e) {
            const int r = i * E1 + e;
            pr1[r] = __builtin_amdgcn_exp2f(fmaf(si[1][r], c, -m));
            l4[r & 3] += pr1[r];
          }
          if (i == NPV / 2 - 1) {
            dropout(pr1, 1, t - 1);
            pack(pr1, 1);
          }
        } else {
#pragma unroll
          for (int e = 0; e < EM; ++e) {
            const int x = (i - NPV / 2) * EM + e;
            mx = fmaxf(mx, so[x >> 4][x & 15]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (i + 1 < NPV) cur = nxt;
      }
    }
    l += (l4[0] + l4[1]) + (l4[2] + l4[3]);
    // rescale decision for S_t (after the PV of tile t-1, which used the old max)
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
    mx = fmaxf(mx, fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]))) * c;
    if (__builtin_amdgcn_ballot_w64(mx > m + kRescaleThr)) {
      const float mn = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      l *= alpha;
#pragma unroll
      for (int i = 0; i < DT; ++i) o[i] *= alpha;
      m = mn;
    }
  };
  // exp / sum / dropout / pack of both sub-tiles of S_{t-1} (drain step, no overlap)
  auto finish = [&](const f32x16 (&si)[2], int t) __attribute__((always_inline)) {
    float l4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      float pr[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        pr[r] = __builtin_amdgcn_exp2f(fmaf(si[kt][r], c, -m));
        l4[r & 3] += pr[r];
      }
      dropout(pr, kt, t);
      pack(pr, kt);
    }
    l += (l4[0] + l4[1]) + (l4[2] + l4[3]);
  };
  // O += V_{t}^T P_{t}^T (V^T fragment one step ahead)
  auto pv = [&](int t) __attribute__((always_inline)) {
    v8 cur = vread(t, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int kt = i / (2 * DT), s2 = (i / DT) & 1, dt = i % DT;
      v8 nxt;
      if (i + 1 < NPV) nxt = vread(t, (i + 1) / (2 * DT), ((i + 1) / DT) & 1, (i + 1) % DT);
      o[dt] = MF<T>::mma(cur, pk[kt][s2], o[dt]);
      if (i + 1 < NPV) cur = nxt;
    }
  };
  auto drain = [&](f32x16 (&si)[2], int t) __attribute__((always_inline)) {  // PV of the wave's last tile t-1
    finish(si, t - 1);
    pv(t - 1);
  };
  auto ring_end = [&]() __attribute__((always_inline)) {
    wait_vm0();
    __builtin_amdgcn_s_barrier();
  };

  if (N > 0) issue(0, 0);
  wait_vm0();
  __builtin_amdgcn_s_barrier();
  // t = 0: QK only
  if (N > 1) issue(1, 0);
  if (N > 0) issue(0, 1);
  if (nact > 0) {
    qk(sa, 0);
    if (0 >= n_int) mask(sa, 0);
    decide(sa);
  }
  ring_end();
  int t = 1;
  // interior tiles, two per trip (S alternates between the named buffers sa / sb)
  for (; t + 1 < n_int; t += 2) {
    if (t + 1 < N) issue(t + 1, 0);
    issue(t, 1);
    steady(sa, sb, t, false);
    ring_end();
    if (t + 2 < N) issue(t + 2, 0);
    issue(t + 1, 1);
    steady(sb, sa, t + 1, false);
    ring_end();
  }
  // pending S in sa; remaining tiles (edge / drain / idle), one per trip with a copy back to sa
  for (; t < N; ++t) {
    if (t + 1 < N) issue(t + 1, 0);
    issue(t, 1);
    if (t < nact) {
      steady(sa, sb, t, t >= n_int);
      sa[0] = sb[0];
      sa[1] = sb[1];
    } else if (t == nact) {
      drain(sa, t);
    }
    ring_end();
  }
  if (nact == N && N > 0) drain(sa, N);

  // ---- epilogue (as attn_fwd_mfma_k)
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  T* orow = out + ((long)b * T_ + min(qi, T_ - 1)) * (long)H * HD + (long)h * HD;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int gq = 0; gq < 4; gq += 2) {
      uint32_t ax = pack2<T>(o[dt][4 * gq + 0] * inv, o[dt][4 * gq + 1] * inv);
      uint32_t ay = pack2<T>(o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv);
      uint32_t bx = pack2<T>(o[dt][4 * gq + 4] * inv, o[dt][4 * gq + 5] * inv);
      uint32_t by = pack2<T>(o[dt][4 * gq + 6] * inv, o[dt][4 * gq + 7] * inv);
      const auto rx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
      ax = rx[0]; bx = rx[1]; ay = ry[0]; by = ry[1];
      if (qi < T_) *reinterpret_cast<uint4*>(orow + dt * 32 + 8 * gq + 8 * hh) = uint4{ax, ay, bx, by};
    }
  if (qi < T_ && hh == 0) lse[((long)b * H + h) * T_ + qi] = m + log2f(lt);
}

bool attn_mfma_head_dim(int hd) { return hd == 64 || hd == 128; }

// forward tiling: 64-key tiles, 2-slot ring, 2 workgroups per CU; for hd 64 with dropout on grids
// of >= 2048 workgroups 32-key tiles with up to 3 workgroups per CU (GPT2-774M B=24 0.179 ->
// 0.163 ms: the hash work wants the third co-resident workgroup).  Dropped: 32-key tiles with a
// 3-slot ring, two 32-query blocks per wave (slower on every shape, profiles/r3/attn_fwd_qb2.md).
static bool fwd_small_tiles(int hd, float p, long nwg) { return hd == 64 && p > 0.f && nwg >= 2048; }

void attn_fwd_mfma(DType dt, const void* qkv, void* o, float* lse, int B, int T_, int H, int G, int hd, bool causal,
                   float p, uint64_t seed, uint64_t offset, uint32_t* keep_mask, hipStream_t s) {
  const uint32_t thr = drop_threshold16(p);
  const float ik = drop_inv_keep(p);
  const bool small = fwd_small_tiles(hd, p, (long)((T_ + FWD_BQ - 1) / FWD_BQ) * H * B);
  const char* xm_env = getenv("BLLM_ATT_XCD");
  const bool xmap = xm_env && xm_env[0] == '1' && (B * G) % 8 == 0;
  const char* pp_env = getenv("BLLM_ATT_PP");
  if (pp_env && pp_env[0] == '3') {
#define LAUNCH_SP(TT, HDD)                                                                                   \
  do {                                                                                                        \
    const dim3 grid(((T_ + 127) / 128) * H * B), block(256);                                                  \
    const int lds = 4 * 64 * HDD * 2;                                                                         \
    if (p > 0.f)                                                                                              \
      hipLaunchKernelGGL((attn_fwd_sp_k<TT, HDD, true>), grid, block, lds, s, (const TT*)qkv, (TT*)o, lse, T_, \
                         H, G, B, causal, thr, ik, seed, offset, keep_mask);                                  \
    else                                                                                                      \
      hipLaunchKernelGGL((attn_fwd_sp_k<TT, HDD, false>), grid, block, lds, s, (const TT*)qkv, (TT*)o, lse,    \
                         T_, H, G, B, causal, thr, ik, seed, offset, nullptr);                                \
  } while (0)
    if (dt == DType::BF16) {
      if (hd == 128) LAUNCH_SP(bf16_t, 128); else LAUNCH_SP(bf16_t, 64);
    } else {
      if (hd == 128) LAUNCH_SP(f16_t, 128); else LAUNCH_SP(f16_t, 64);
    }
#undef LAUNCH_SP
    return;
  }
  if (pp_env && (pp_env[0] == '1' || pp_env[0] == '2')) {
    static unsigned long long* dbuf = nullptr;
    unsigned long long* dbg = nullptr;
    if (pp_env[0] == '2') {
      if (!dbuf) (void)hipMalloc(&dbuf, 16 * 8 * 64 * 8);
      (void)hipMemsetAsync(dbuf, 0, 16 * 8 * 64 * 8, s);
      dbg = dbuf;
    }
#define LAUNCH_PP(TT, HDD)                                                                                   \
  do {                                                                                                        \
    const dim3 grid(((T_ + 255) / 256) * H * B), block(512);                                                  \
    const int lds = 6 * 64 * HDD * 2;                                                                         \
    static const bool at0 = hipFuncSetAttribute((const void*)attn_fwd_pp_k<TT, HDD, true>,                   \
                                                hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess; \
    static const bool at1 = hipFuncSetAttribute((const void*)attn_fwd_pp_k<TT, HDD, false>,                  \
                                                hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess; \
    (void)at0;                                                                                                \
    (void)at1;                                                                                                \
    if (p > 0.f)                                                                                              \
      hipLaunchKernelGGL((attn_fwd_pp_k<TT, HDD, true>), grid, block, lds, s, (const TT*)qkv, (TT*)o, lse, T_, \
                         H, G, B, causal, thr, ik, seed, offset, keep_mask, dbg);                             \
    else                                                                                                      \
      hipLaunchKernelGGL((attn_fwd_pp_k<TT, HDD, false>), grid, block, lds, s, (const TT*)qkv, (TT*)o, lse,    \
                         T_, H, G, B, causal, thr, ik, seed, offset, nullptr, dbg);                           \
  } while (0)
    if (dt == DType::BF16) {
      if (hd == 128) LAUNCH_PP(bf16_t, 128); else LAUNCH_PP(bf16_t, 64);
    } else {
      if (hd == 128) LAUNCH_PP(f16_t, 128); else LAUNCH_PP(f16_t, 64);
    }
#undef LAUNCH_PP
    if (dbg) {  // per-phase cycle summary of the first 16 workgroups (debug)
      static unsigned long long h[16 * 8 * 64];
      (void)hipMemcpyAsync(h, dbg, sizeof(h), hipMemcpyDeviceToHost, s);
      (void)hipStreamSynchronize(s);
      for (int wg = 0; wg < 16; wg += 5)
        for (int w = 0; w < 8; w += 4) {
          const unsigned long long* t = h + (wg * 8 + w) * 64;
          fprintf(stderr, "pp-stamp wg %d w %d:", wg, w);
          for (int i = 1; i < 64 && t[i]; ++i) fprintf(stderr, " %lld", (long long)(t[i] - t[i - 1]));
          fprintf(stderr, "\n");
        }
    }
    return;
  }
#define LAUNCH_V(TT, HDD, BK, NB, OC)                                                                      \
  do {                                                                                                        \
    const int lds = NB * 2 * BK * HDD * 2;                                                                    \
    const dim3 grid(((T_ + FWD_BQ - 1) / FWD_BQ) * H * B), block(256);                                        \
    if (p > 0.f)                                                                                              \
      hipLaunchKernelGGL((attn_fwd_mfma_k<TT, HDD, true, BK, NB, OC>), grid, block, lds, s,          \
                         (const TT*)qkv, (TT*)o, lse, T_, H, G, B, causal, thr, ik, seed, offset, keep_mask, xmap); \
    else                                                                                                      \
      hipLaunchKernelGGL((attn_fwd_mfma_k<TT, HDD, false, BK, NB, OC>), grid, block, lds, s,         \
                         (const TT*)qkv, (TT*)o, lse, T_, H, G, B, causal, thr, ik, seed, offset, nullptr, xmap); \
  } while (0)
#define LAUNCH(TT, HDD)                                                                                       \
  do {                                                                                                        \
    if (small) LAUNCH_V(TT, HDD, 32, 2, 3);                                                                   \
    else LAUNCH_V(TT, HDD, 64, 2, 2);                                                                         \
  } while (0)
  if (dt == DType::BF16) {
    if (hd == 128) LAUNCH(bf16_t, 128); else LAUNCH(bf16_t, 64);
  } else {
    if (hd == 128) LAUNCH(f16_t, 128); else LAUNCH(f16_t, 64);
  }
#undef LAUNCH
#undef LAUNCH_V
}

}  // namespace bllm
