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
                                                          uint64_t doff, uint32_t* __restrict__ kmask, int xmap) {
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
  // (b, h) and (xmap 1) the query heads of one kv head run on one XCD / L2 (common.h)
  const int nqb = (T_ + BQ - 1) / BQ;
  const int lin = blockIdx.x, nbh = H * B_;
  int qbi, bh;
  attn_wg_order(lin, nbh, H / G, xmap, qbi, bh);
  const int h = bh % H, b = bh / H;
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
              s[u][kt][r] = k0b ? s[u][kt][r] : 0.f;
              s[u][kt][r + 1] = k1b ? s[u][kt][r + 1] : 0.f;
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
              s[u][kt][r] = kb_ ? s[u][kt][r] : 0.f;
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
    // dropout's 1 / keep applied once here instead of to every kept probability
    const float inv = lt > 0.f ? (DROP ? inv_keep : 1.f) / lt : 0.f;
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

bool attn_mfma_head_dim(int hd) { return hd == 64 || hd == 128; }

// forward tiling: 64-key tiles, 2-slot ring, 2 workgroups per CU; for hd 64 on grids of >= 2048
// workgroups 32-key tiles with up to 3 workgroups per CU (GPT2-774M B=24 with dropout 0.179 ->
// 0.163 ms: the hash work wants the third co-resident workgroup; round 6, after the XCD order:
// Llama-3.2-1B B=24 without dropout 658 -> 686 TF/s, GPT-2 without dropout unchanged,
// profiles/r6/attn/smalltiles/).  Dropped: 32-key tiles with a 3-slot ring, two 32-query blocks
// per wave (slower on every shape, profiles/r3/attn_fwd_qb2.md).
static bool fwd_small_tiles(int hd, float p, long nwg) {
  (void)p;
  return hd == 64 && nwg >= 2048;
}

void attn_fwd_mfma(DType dt, const void* qkv, void* o, float* lse, int B, int T_, int H, int G, int hd, bool causal,
                   float p, uint64_t seed, uint64_t offset, uint32_t* keep_mask, hipStream_t s) {
  const uint32_t thr = drop_threshold16(p);
  const float ik = drop_inv_keep(p);
  const bool small = fwd_small_tiles(hd, p, (long)((T_ + FWD_BQ - 1) / FWD_BQ) * H * B);
  // XCD-aware workgroup order when the (batch, kv head) groups split evenly over the 8 XCDs
  const int xmap = attn_xcd_order_ok(B * H, H / G) ? 1 : 0;
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
