// LoRA low-rank path on CDNA4 matrix cores (v_mfma_f32_16x16x32_{bf16,f16}).
//
// Replaces reference lora.py:24-26,45-46 (``x @ A @ B * scaling`` added to every nn.Linear,
// LinearWithLoRA) and its autograd.  A fused linear group (Q/K/V, gate/up, or a single
// projection) has up to LORA_MAX_MEMBERS LoRA members m with A_m [in, r_m], B_m [r_m, out_m];
// member m owns the column window [c0_m, c0_m + out_m) of the group's output.  Three kernels
// cover forward and backward (s = alpha / r):
//
//   lora_down   T[:, off_m : off_m + r_m] = X[:, c0_m : c0_m + len_m] . W_m^T
//               fwd: t = x . A  (W = packed A^T, all members read the whole x)
//               bwd: u = dy . B^T (W = B itself, member m reads its dy window)
//   lora_up     Y[:, c0_m : c0_m + len_m] += s . T[:, off_m : off_m + r_m] . U_m
//               fwd: y += s t B  (U = B);  bwd: dx += s u A^T (U = A^T)
//   lora_wgrad  G_m = s . P[:, a-window]^T . Q[:, b-window]   (reduction over the N tokens)
//               dB = s t^T dy,  dA = s x^T u — written (or accumulated) straight into the
//               unit's flat gradient in its dtype; deterministic (fixed-order split-N partials).
//               Members that read the same Q window (every dA of a group: all read x) are
//               merged by the binding into one of rank sum r_m <= 64, so x is streamed once;
//               its 16-column tiles carry their own output pointers (gt).
//
// All three are HBM-bound (the rank is 8-64): x / dy / y are streamed exactly once per kernel
// with 16-byte lane accesses; the small operands (A, B, t, u) stay L2-resident.
#include "api.h"

namespace bllm {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <typename T> struct MF16;
template <> struct MF16<bf16_t> {
  static __device__ __forceinline__ f32x4 mma(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
};
template <> struct MF16<f16_t> {
  static __device__ __forceinline__ f32x4 mma(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
  }
};

__device__ __forceinline__ s16x8 ld8(const void* p) { return *reinterpret_cast<const s16x8*>(p); }

template <typename T> __device__ __forceinline__ short bits_of(float v) {
  const T h = from_f<T>(v);
  return __builtin_bit_cast(short, h);
}
template <typename T> __device__ __forceinline__ float from_bits(short b) {
  return to_f(__builtin_bit_cast(T, b));
}

// --------------------------------------------------------------------------- lora_down
// Block = 4 waves on 64 rows; the waves split K (wave w takes k-steps w, w+4, ...; two per trip:
// 8 x loads in flight per lane) and each runs the block's 4 row tiles against ONE W fragment per
// column tile and k-step, so W (the packed A^T / B, nt*16 columns) crosses L2 -> CU once per 64
// rows.  (Round 4's kernel did 16 rows per block: at nt = 2-3 (gate/up, QKV) it moved 2-3x more
// W than x bytes and ran at 2.2-2.9 TB/s of x; this one 3.2-5.2 TB/s, tools/bench_lora.py,
// profiles/r5/lora_kernels/.)  MFMA: A = X rows (lane: X[row l&15][k 8(l>>4)..+8], one 16-B load),
// B[k][col] = W[col][k] (W rows are k-contiguous -> one 16-B load per column tile).  The four
// partial [64 x cols] tiles meet in (dynamic) LDS and are summed in a fixed order.
template <typename T, int NTM>
__global__ __launch_bounds__(256) void lora_down4_k(LoraDownArgs a, int N) {
  constexpr int NW = 4, RT = 4, ROWS = 16 * RT;  // NTM: max column tiles over the launch's chunks
  extern __shared__ float red4[];  // [NW][ROWS][cols + 1]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ch = blockIdx.y;
  const int nt = a.nt[ch], cols = nt * 16, ldr = cols + 1;
  const long row0 = (long)blockIdx.x * ROWS;
  const T* xs[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    // rows past the token count read row N-1 (never stored)
    const long xr = row0 + rt * 16 + (lane & 15) < N ? row0 + rt * 16 + (lane & 15) : N - 1;
    xs[rt] = (const T*)a.x + xr * a.ldx + a.c0[ch] + 8 * (lane >> 4);
  }
  const T* w = (const T*)a.w[ch] + (long)(lane & 15) * a.ldw[ch] + 8 * (lane >> 4);
  const long wstep = 16 * a.ldw[ch];
  f32x4 acc[RT][NTM];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NTM; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nks = a.len[ch] >> 5;
  int ks = wave;
  for (; ks + NW < nks; ks += 2 * NW) {  // two k-steps per trip: 8 x loads in flight per lane
    s16x8 xa[2][RT];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) xa[u][rt] = ld8(xs[rt] + (ks + u * NW) * 32);
#pragma unroll
    for (int t = 0; t < NTM; ++t) {
      if (t < nt) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const s16x8 wb = ld8(w + t * wstep + (ks + u * NW) * 32);
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) acc[rt][t] = MF16<T>::mma(xa[u][rt], wb, acc[rt][t]);
        }
      }
    }
  }
  for (; ks < nks; ks += NW) {
    s16x8 xa[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) xa[rt] = ld8(xs[rt] + ks * 32);
#pragma unroll
    for (int t = 0; t < NTM; ++t) {
      if (t < nt) {
        const s16x8 wb = ld8(w + t * wstep + ks * 32);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][t] = MF16<T>::mma(xa[rt], wb, acc[rt][t]);
      }
    }
  }
  // C layout: lane holds C[row 4(l>>4)+i][col l&15] of each 16 x 16 tile
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NTM; ++t)
      if (t < nt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          red4[(wave * ROWS + rt * 16 + 4 * (lane >> 4) + i) * ldr + t * 16 + (lane & 15)] = acc[rt][t][i];
  __syncthreads();
  T* out = (T*)a.out + row0 * a.ldo + a.ocol[ch];
  for (int e = threadIdx.x; e < ROWS * cols; e += NW * 64) {
    const int r = e / cols, c = e - r * cols;
    if (row0 + r >= N) continue;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += red4[(q * ROWS + r) * ldr + c];
    out[(long)r * a.ldo + c] = from_f<T>(v * a.scale);
  }
  if (ch == 0 && a.zpad > 0) {  // zero columns [R, R + zpad): the alignment pad of a K-augmented row
    T* pad = (T*)a.out + row0 * a.ldo + a.R;
    for (int e = threadIdx.x; e < ROWS * a.zpad; e += NW * 64) {
      const int r = e / a.zpad, c = e - r * a.zpad;
      if (row0 + r < N) pad[(long)r * a.ldo + c] = from_f<T>(0.f);
    }
  }
}

// --------------------------------------------------------------------------- lora_up
// out[:, c0 + c] = base[:, c0 + c] + bias[c0 + c] + s . (t[:, toff : toff + r] . U)[:, c]
// (base / bias optional; base may alias out).  Used write-only ahead of a beta=1 GEMM, so the
// low-rank update rides on the GEMM's C read instead of a separate read-modify-write pass.
// Block = `rows` (64-256) rows x 128 columns of one member window; each of the 4 waves walks its rows in
// 16-row tiles reusing U's [r x 128] slice, staged once per block in LDS as [col][r] (one 16-B
// read per A fragment).  The product is formed transposed, Y^T tile [16 cols x 16 rows] =
// U^T . T^T (B fragment = a 16-B global read of a t row); the fp32 tile is re-laid through a
// per-wave LDS buffer so every lane stores 16 contiguous bytes.
template <typename T>
__global__ __launch_bounds__(256) void lora_up_k(LoraUpArgs a, int rows, int N) {
  constexpr int BN = 128, RP = 64 + 8, EP = BN + 4;
  __shared__ __attribute__((aligned(16))) short us[BN * RP];
  __shared__ __attribute__((aligned(16))) float eps_[4 * 16 * EP];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int m = blockIdx.z;
  const int r = a.r[m], len = a.len[m];
  const int cb = blockIdx.y * BN;
  if (cb >= len) return;
  const T* U = (const T*)a.u[m];
  const long su_j = a.su_j[m], su_c = a.su_c[m];
  float* ep = eps_ + wave * 16 * EP;
  const int c8 = (lane & 15) * 8;
  const bool col_ok = cb + c8 + 8 <= len;
  const T* bias = (const T*)a.bias;
  VecN<T, 8> bb;
  if (bias && col_ok) bb = ldv<T, 8>(bias + a.c0[m] + cb + c8);
  const s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j0 = 0; j0 < r; j0 += 64) {  // ranks > 64 in 64-wide LDS passes (rare: r <= 64 is one)
    const int rc = r - j0 < 64 ? r - j0 : 64;
    if (j0) __syncthreads();
    if (su_c == 1 && (len & 7) == 0) {  // 16-B loads of 8 columns of one U row
      for (int e = threadIdx.x; e < (BN / 8) * rc; e += 256) {
        const int j = e / (BN / 8), c = (e - j * (BN / 8)) * 8;
        s16x8 v = zero;
        if (cb + c < len) v = ld8(U + (long)(j0 + j) * su_j + cb + c);
#pragma unroll
        for (int i = 0; i < 8; ++i) us[(c + i) * RP + j] = v[i];
      }
    } else {
      for (int e = threadIdx.x; e < BN * rc; e += 256) {
        const int c = e / rc, j = e - c * rc;  // r-fastest: coalesced when su_j == 1 (U = A^T)
        short v = 0;
        if (cb + c < len) v = __builtin_bit_cast(short, U[(long)(j0 + j) * su_j + (long)(cb + c) * su_c]);
        us[c * RP + j] = v;
      }
    }
    __syncthreads();
    // the base (or, in a later rank pass, y) rows of a tile are loaded one tile ahead (register
    // double buffer): loaded inside the epilogue, one 4-row group at a time, they left the
    // kernel latency-bound at ~3 TB/s
    VecN<T, 8> bsv[4], bsn[4];
    auto load_base = [&](long r0_, VecN<T, 8> (&dst)[4]) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int row = (lane >> 4) + 4 * p;
        if (col_ok && r0_ + row < N) {
          if (j0) dst[p] = ldv<T, 8>((const T*)a.y + (r0_ + row) * a.ldy + a.c0[m] + cb + c8);
          else if (a.base) dst[p] = ldv<T, 8>((const T*)a.base + (r0_ + row) * a.ldb + a.c0[m] + cb + c8);
        }
      }
    };
    // the tile's t rows (the MFMA B fragments, rc <= 64: at most two 32-deep k-steps) are
    // prefetched a tile ahead too: loaded in front of the MFMAs they left every tile waiting a
    // full load latency
    s16x8 tbv[2], tbn[2];
    auto load_t = [&](long r0_, s16x8 (&dst)[2]) {
      const long tr = r0_ + (lane & 15) < N ? r0_ + (lane & 15) : N - 1;
      const T* t = (const T*)a.t + tr * a.ldt + a.toff[m] + j0;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int kk = 32 * ks + 8 * (lane >> 4);
        dst[ks] = kk < rc ? ld8(t + kk) : zero;  // r % 16 == 0: the upper half of a step may be padding
      }
    };
    load_base((long)blockIdx.x * rows + wave * 16, bsv);
    load_t((long)blockIdx.x * rows + wave * 16, tbv);
    for (int rt = 0; rt < rows / 64; ++rt) {
      const long row0 = (long)blockIdx.x * rows + rt * 64 + wave * 16;
      if (row0 >= N) break;  // wave-uniform: this wave's remaining tiles are past the tokens
      if (rt + 1 < rows / 64 && row0 + 64 < N) {
        load_base(row0 + 64, bsn);
        load_t(row0 + 64, tbn);
      }
      f32x4 acc[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (32 * ks >= rc) break;
        const int kk = 32 * ks + 8 * (lane >> 4);
        const bool live = kk < rc;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const s16x8 ua = live ? *reinterpret_cast<const s16x8*>(&us[(q * 16 + (lane & 15)) * RP + kk]) : zero;
          acc[q] = MF16<T>::mma(ua, tbv[ks], acc[q]);
        }
      }
      // lane holds Y^T[col q*16 + 4(l>>4) + i][row l&15] -> per-wave [16 rows][128 cols] fp32 tile
#pragma unroll
      for (int q = 0; q < 8; ++q)
        *reinterpret_cast<f32x4*>(&ep[(lane & 15) * EP + q * 16 + 4 * (lane >> 4)]) = acc[q];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's tile writes have landed
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int row = (lane >> 4) + 4 * p;
        if (!col_ok || row0 + row >= N) continue;
        const long g = (row0 + row) * a.ldy + a.c0[m] + cb + c8;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(&ep[row * EP + c8]);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(&ep[row * EP + c8 + 4]);
        const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        // later rank pass: bsv holds what the first pass wrote (y)
        const VecN<T, 8> bs = bsv[p];
        VecN<T, 8> o;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float z = a.scale * v[i];
          if (a.base || j0) z += to_f(bs.v[i]);
          if (bias && !j0) z += to_f(bb.v[i]);
          o.v[i] = from_f<T>(z);
        }
        stv<T, 8>((T*)a.y + g, o);
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) bsv[p] = bsn[p];
      tbv[0] = tbn[0];
      tbv[1] = tbn[1];
      __builtin_amdgcn_wave_barrier();  // tile reads done before the next tile's writes
    }
  }
}

// --------------------------------------------------------------------------- lora_wgrad
// G[b][a] = s . sum_n Q[n][qb + b] . P[n][pa + a]  for b < len (64 per block), a < r.
// The token dimension is the MFMA K.  64-token chunks of Q [64 n x 64 b] and P [64 n x r] are
// stored row-major into LDS with 16-B writes and consumed column-major through the hardware
// transpose read (ds_read_b64_tr_b16: a 16-lane group gets 4 rows x 16 columns delivered
// column-major), two reads per 8-token fragment.  The next chunk's global loads are issued
// before the current chunk's MFMAs.  Split-N over gridDim.y; with S > 1 each split writes an
// fp32 partial G that lora_reduce sums in a fixed order (deterministic, no atomics).
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x8 tr_frag(const short* base, int stride) {
  // rows 0..3 and 4..7 of an 8-row column block -> the 8 k-elements of a 16x16x32 fragment
  const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
  const s16x4 r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 4 * stride));
  return s16x8{r1[0], r1[1], r1[2], r1[3], r2[0], r2[1], r2[2], r2[3]};
}

template <typename T, typename OT>
__global__ __launch_bounds__(256) void lora_wgrad_k(LoraWgradArgs a, int N) {
  constexpr int NP = 64 + 8;  // padded row (144 B) of the [n][col] images
  __shared__ __attribute__((aligned(16))) short qs[64 * NP];
  __shared__ __attribute__((aligned(16))) short ps[64 * NP];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int m = 0, bx = blockIdx.x;
  while (m + 1 < a.n && bx >= a.nblk[m]) { bx -= a.nblk[m]; ++m; }
  const int r = a.r[m], len = a.len[m];
  const int b0 = bx * 64;
  const int S = gridDim.y, split = blockIdx.y;
  const int nchunks = (N + 63) / 64;
  const int c_lo = (int)((long)nchunks * split / S), c_hi = (int)((long)nchunks * (split + 1) / S);
  const T* Q = (const T*)a.q + a.qb[m];
  const T* P = (const T*)a.p + a.pa[m];
  const int nt = r >> 4;
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int sn = threadIdx.x >> 3, sc = (threadIdx.x & 7) * 8;  // staging: token sn (+32), 8 columns
  const bool q_ok = b0 + sc + 8 <= len, p_ok = sc < r;
  const s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  s16x8 qv[2], pv[2];
  auto load = [&](int ck) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const long n = (long)ck * 64 + sn + 32 * h;
      const bool n_ok = n < N;  // tail chunk of an N % 64 != 0 batch: zero tokens
      qv[h] = q_ok && n_ok ? ld8(Q + n * a.ldq + b0 + sc) : zero;
      pv[h] = p_ok && n_ok ? ld8(P + n * a.ldp + sc) : zero;
    }
  };
  // tr-read addresses: lane 4q+p of each 16-lane group -> row q, columns 4p..4p+3 of the block
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg = lane >> 4;
  if (c_lo < c_hi) load(c_lo);
  for (int ck = c_lo; ck < c_hi; ++ck) {
    __syncthreads();  // previous chunk's fragment reads are done
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      *reinterpret_cast<s16x8*>(&qs[(sn + 32 * h) * NP + sc]) = qv[h];
      *reinterpret_cast<s16x8*>(&ps[(sn + 32 * h) * NP + sc]) = pv[h];
    }
    if (ck + 1 < c_hi) load(ck + 1);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int n = ks * 32 + 8 * tg + tq;
      const s16x8 qa = tr_frag(&qs[n * NP + wave * 16 + 4 * tp], NP);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < nt) acc[t] = MF16<T>::mma(qa, tr_frag(&ps[n * NP + t * 16 + 4 * tp], NP), acc[t]);
    }
  }
  // lane holds G[b = b0 + 16*wave + 4(l>>4) + i][a = 16t + (l&15)]; column tile t of member m
  // goes to gt[m][t] (a merged member spans several output matrices, 16 columns each at least)
  const long sa = a.sa[m], sb = a.sb[m];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t >= nt) continue;
    OT* gtile = (OT*)a.gt[m][t];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = b0 + wave * 16 + 4 * (lane >> 4) + i, ac = lane & 15;
      if (b >= len) continue;
      const float v = acc[t][i] * a.scale;
      if (S > 1) {  // dense [r][len] partial
        a.part[(long)split * a.part_ld + a.part_off[m] + (long)(t * 16 + ac) * len + b] = v;
      } else {
        const long o = (long)ac * sa + (long)b * sb;
        gtile[o] = from_f<OT>(a.accumulate ? to_f(gtile[o]) + v : v);
      }
    }
  }
}

// g_m[e] (+)= sum_s part[s][off_m + e] for every member, one launch, fixed summation order
template <typename OT>
__global__ __launch_bounds__(256) void lora_reduce_k(LoraWgradArgs a, int S, long total) {
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    int m = 0;
    while (m + 1 < a.n && e >= a.part_off[m + 1]) ++m;
    const long o = e - a.part_off[m];
    const int aa = (int)(o / a.len[m]);
    const long b = o - (long)aa * a.len[m];
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += a.part[(long)s * a.part_ld + e];
    OT* g = (OT*)a.gt[m][aa >> 4] + (long)(aa & 15) * a.sa[m] + b * a.sb[m];
    *g = from_f<OT>(a.accumulate ? to_f(*g) + v : v);
  }
}

// P[off_m + j][k] = A_m[k][j]: pack the members' A [K, r_m] into one k-contiguous [R, K] operand
template <typename T>
__global__ __launch_bounds__(256) void lora_pack_t_k(LoraPackArgs a, int K) {
  const int m = blockIdx.y;
  const int r = a.r[m];
  const T* A = (const T*)a.a[m];
  T* P = (T*)a.out + (long)a.off[m] * K;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < (long)K * r; e += (long)gridDim.x * 256) {
    const long k = e / r;
    const int j = (int)(e - k * r);
    P[(long)j * K + k] = A[e];
  }
}

// The B block of a K-augmented weight: [W | Bd^T] (forward, dst row-major [out, K + R] at column K)
// or [W^T ; Bd] (the dX GEMM's transposed operand, at row K).  Every (row, j) of the [out, R]
// block is written -- B_m^T inside member m's rows x rank columns, 0 elsewhere -- the unit-stride
// index fastest.
template <typename T>
__global__ __launch_bounds__(256) void lora_block_k(LoraBlockArgs a) {
  const long total = (long)a.rows * a.R;
  const bool row_fast = a.s_row == 1;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int row = row_fast ? (int)(e % a.rows) : (int)(e / a.R);
    const int j = row_fast ? (int)(e / a.rows) : (int)(e % a.R);
    T v = from_f<T>(0.f);
    for (int m = 0; m < a.n; ++m) {
      const int rr = row - a.c0[m], jj = j - a.off[m];
      if (rr >= 0 && rr < a.len[m] && jj >= 0 && jj < a.r[m]) v = ((const T*)a.b[m])[(long)jj * a.ldb[m] + rr];
    }
    ((T*)a.dst)[(long)row * a.s_row + (long)j * a.s_j] = v;
  }
}

}  // namespace

// --------------------------------------------------------------------------- lora_head_bwd
// The LoRA head's two rank-16 products of one logits-gradient chunk dl [R, V] in ONE pass over dl
// (both used to stream it: u = dl B^T on hipBLASLt, dB = (s t)^T dl on lora_wgrad):
//   gpart[ry][j][c] = sum_{n in rows of ry} st[n][j] dl[n][c]      (dB partial per row range)
//   upart[cx][n][j] = sum_{c in slab cx} dl[n][c] B[j][c]          (u partial per column slab)
// A workgroup owns a slab of up to 1,024 columns (16 sub-slabs of 64) and a row range, walked in
// 64-row chunks; B's [16 x 1,024] slab is staged in LDS once, and per (chunk, sub-slab) the dl tile
// [64 x 64] (4 tiles in flight in registers) is staged in LDS (double-buffered, one barrier), then
// wave w adds its 16 columns of dB (A = st^T, B = dl, both transposed reads, K = rows) and its 16
// rows of u (A = dl rows, B = B rows, K = columns).  lhb_usum_k / lora_reduce finish both sums in
// a fixed order (deterministic).
constexpr int LHB_SUB = 64, LHB_NSUB = 16, LHB_ROWS = 64;
constexpr int LHB_DS = LHB_SUB * 2 + 16;  // bytes per row of a dl tile (padded)
constexpr int LHB_SS = 32;                // bytes per row of the st tile
constexpr int LHB_BS = LHB_SUB * LHB_NSUB * 2 + 16;  // bytes per row of the staged B slab (padded)

__device__ __forceinline__ s16x8 lhb_tr(const char* tile, int stride, int col_byte, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const char* a = tile + (8 * g + q) * stride + col_byte + 8 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * stride));
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <typename T, int D>
__global__ __launch_bounds__(256) void lora_head_bwd_k(const T* __restrict__ dl, long ldl, const T* __restrict__ st,
                                                       long ldst, const T* __restrict__ Bm, long ldb,
                                                       float* __restrict__ gpart, float* __restrict__ upart, int R,
                                                       int V, int rows_per) {
  __shared__ __attribute__((aligned(16))) char Dt[2][LHB_ROWS * LHB_DS];
  // the slab's B [16 x 1,024] stays in LDS for the whole row range (staged once)
  __shared__ __attribute__((aligned(16))) char Bs[16 * LHB_BS];
  __shared__ __attribute__((aligned(16))) char St[LHB_ROWS * LHB_SS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c0 = blockIdx.x * LHB_SUB * LHB_NSUB;
  const int nsub = (V - c0) / LHB_SUB < LHB_NSUB ? (V - c0) / LHB_SUB : LHB_NSUB;
  // every slab runs all 16 sub-slabs (the last slab's missing ones on zero tiles: its dB columns are
  // not stored, its u terms are 0): no data-dependent control flow around the MFMA accumulators, and
  // the register set of iteration (chunk, sub) is sub % D at compile time
  constexpr int nsubP = LHB_NSUB;
  const int r0 = blockIdx.y * rows_per, r1 = r0 + rows_per < R ? r0 + rows_per : R;
  const s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  // staging roles: dl tile rows dr, dr + 32 at 16-B chunk dc; st row sr half sh (threads < 128)
  const int dr = tid >> 3, dc = (tid & 7) * 8, sr = tid >> 1, sh = tid & 1;
  f32x4 accB[LHB_NSUB];
#pragma unroll
  for (int k = 0; k < LHB_NSUB; ++k) accB[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 pd0[D], pd1[D], ps = zero;
  for (int e = tid; e < 16 * LHB_NSUB * (LHB_SUB / 8); e += 256) {
    const int j = e / (LHB_NSUB * LHB_SUB / 8), c = (e - j * (LHB_NSUB * LHB_SUB / 8)) * 8;
    *reinterpret_cast<s16x8*>(Bs + j * LHB_BS + 2 * c) = c < nsub * LHB_SUB ? ld8(Bm + (long)j * ldb + c0 + c) : zero;
  }
  // Loads are raw buffer loads on descriptors bounded to this workgroup's rows: a row past r1 (and
  // a padded sub-slab, sent to an offset past every bound) reads as 0 with no branch, so the
  // compiler can keep the D pieces in flight (exec-masked loads made it drain vmcnt to 0).
  constexpr int OOB = 0x7ffffff0;
  const int nrow = r1 > r0 ? r1 - r0 : 0;
  const __amdgpu_buffer_rsrc_t rd =
      __builtin_amdgcn_make_buffer_rsrc((void*)(dl + (long)r0 * ldl), (short)0, (int)((long)nrow * ldl * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(st + (long)r0 * ldst), (short)0, (int)((long)nrow * ldst * 2), 0x00020000);
  const int half_off = (int)(32L * ldl * 2);  // rows dr + 32
  // load cursor: (lrow, lsub) of the next piece to fetch, D iterations ahead of the MFMAs, as
  // running byte offsets (not per-sub addresses, which the unrolled loop would keep live)
  int lsub = 0;
  int od = (int)(((long)dr * ldl + c0 + dc) * 2);
  const int dstep = (int)(((long)LHB_ROWS * ldl - (long)nsubP * LHB_SUB) * 2);
  auto bld = [](const __amdgpu_buffer_rsrc_t& r, int off, int soff) {
    return __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 0));
  };
  auto load = [&](int k) {  // this thread's pieces of the cursor's (chunk, sub-slab) into register set k
    const bool in = lsub < nsub;
    pd0[k] = bld(rd, in ? od : OOB, 0);
    pd1[k] = bld(rd, in ? od + half_off : OOB, 0);
    od += LHB_SUB * 2;
    if (++lsub == nsubP) { lsub = 0; od += dstep; }
  };
  auto load_st = [&](int row) {
    if (tid < 128) ps = bld(rs, (int)(((long)(row - r0 + sr) * ldst + 8 * sh) * 2), 0);
  };
#pragma unroll
  for (int k = 0; k < D; ++k) load(k);
  load_st(r0);
  int par = 0;
  for (int row = r0; row < r1; row += LHB_ROWS) {
    // st rows of this chunk (the previous chunk's readers are past its closing barrier)
    if (tid < 128) *reinterpret_cast<s16x8*>(St + sr * LHB_SS + 16 * sh) = ps;
    load_st(row + LHB_ROWS);
    f32x4 accU = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sub = 0; sub < LHB_NSUB; ++sub) {
      {
        const int k = sub % D;
        {
          *reinterpret_cast<s16x8*>(Dt[par] + dr * LHB_DS + dc * 2) = pd0[k];
          *reinterpret_cast<s16x8*>(Dt[par] + (32 + dr) * LHB_DS + dc * 2) = pd1[k];
          __syncthreads();
        }
        load(k);
        {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            // dB: [16 j x 16 cols of wave w] += st^T [16 x 32 rows] . dl [32 rows x 16 cols]
            const s16x8 a = lhb_tr(St + ks * 32 * LHB_SS, LHB_SS, 0, lane);
            const s16x8 b = lhb_tr(Dt[par] + ks * 32 * LHB_DS, LHB_DS, 32 * w, lane);
            accB[sub] = MF16<T>::mma(a, b, accB[sub]);
            // u: [16 rows of wave w x 16 j] += dl [16 rows x 32 cols] . B^T [32 cols x 16 j]
            const int k8 = 32 * ks + 8 * (lane >> 4);
            const s16x8 ua = *reinterpret_cast<const s16x8*>(Dt[par] + (16 * w + (lane & 15)) * LHB_DS + 2 * k8);
            const s16x8 ub = *reinterpret_cast<const s16x8*>(Bs + (lane & 15) * LHB_BS + 2 * (sub * LHB_SUB + k8));
            accU = MF16<T>::mma(ua, ub, accU);
          }
          par ^= 1;
        }
      }
    }
    // u partial of this slab: lane holds C[row 16w + 4(l>>4) + i][j = l&15]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = row + 16 * w + 4 * (lane >> 4) + i;
      if (rr < r1) upart[((long)blockIdx.x * R + rr) * 16 + (lane & 15)] = accU[i];
    }
    __syncthreads();  // St is rewritten by the next chunk
  }
  // dB partial of this row range: lane holds C[j = 4(l>>4) + i][col = 16w + (l&15)] per sub-slab
#pragma unroll
  for (int sub = 0; sub < LHB_NSUB; ++sub)
    if (sub < nsub)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        gpart[((long)blockIdx.y * 16 + 4 * (lane >> 4) + i) * V + c0 + sub * LHB_SUB + 16 * w + (lane & 15)] = accB[sub][i];
}

// u[e] = sum over the column slabs of upart[slab][e] (fp32, fixed order), for the ~126 slabs of a
// 128k vocabulary: a workgroup owns 256 outputs, wave w sums slabs w, w + 4, ... (4 loads in flight
// per lane), then wave 0 adds the 4 wave sums in order.
template <typename T>
__global__ __launch_bounds__(256) void lhb_usum_k(const float* __restrict__ upart, T* __restrict__ u, long n,
                                                  int slabs) {
  __shared__ f32x4 red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 256 + 4 * lane;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (e < n) {
    int q = w;
    for (; q + 12 < slabs; q += 16) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(upart + (long)q * n + e);
      const f32x4 b = *reinterpret_cast<const f32x4*>(upart + (long)(q + 4) * n + e);
      const f32x4 c = *reinterpret_cast<const f32x4*>(upart + (long)(q + 8) * n + e);
      const f32x4 d = *reinterpret_cast<const f32x4*>(upart + (long)(q + 12) * n + e);
      acc = acc + a;
      acc = acc + b;
      acc = acc + c;
      acc = acc + d;
    }
    for (; q < slabs; q += 4) acc = acc + *reinterpret_cast<const f32x4*>(upart + (long)q * n + e);
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && e < n) {
    const f32x4 t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    s16x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = bits_of<T>(t[i]);
    *reinterpret_cast<s16x4*>(u + e) = o;
  }
}

// ----------------------------------------------------------------------------- launchers
void lora_block(DType dt, const LoraBlockArgs& a, hipStream_t s) {
  const long total = (long)a.rows * a.R;
  const int g = (int)((total + 255) / 256 < 1024 ? (total + 255) / 256 : 1024);
  if (dt == DType::BF16) hipLaunchKernelGGL(lora_block_k<bf16_t>, dim3(g), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(lora_block_k<f16_t>, dim3(g), dim3(256), 0, s, a);
}

void lora_down(DType dt, const LoraDownArgs& a, int N, hipStream_t s) {
  int max_cols = 16;
  for (int c = 0; c < a.n; ++c) max_cols = max_cols > a.nt[c] * 16 ? max_cols : a.nt[c] * 16;
  const size_t lds = (size_t)4 * 64 * (max_cols + 1) * sizeof(float);
  dim3 grid(ceil_div(N, 64), a.n);
#define LD4(TT, NTM)                                                                                            \
  do {                                                                                                          \
    static const bool attr = hipFuncSetAttribute((const void*)lora_down4_k<TT, NTM>,                           \
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 64 * 65 * 4) == \
                             hipSuccess;                                                                        \
    (void)attr;                                                                                                 \
    hipLaunchKernelGGL((lora_down4_k<TT, NTM>), grid, dim3(256), lds, s, a, N);                                 \
  } while (0)
  const int ntm = max_cols / 16;
  if (dt == DType::BF16) {
    if (ntm == 1) LD4(bf16_t, 1); else if (ntm == 2) LD4(bf16_t, 2); else if (ntm == 3) LD4(bf16_t, 3); else LD4(bf16_t, 4);
  } else {
    if (ntm == 1) LD4(f16_t, 1); else if (ntm == 2) LD4(f16_t, 2); else if (ntm == 3) LD4(f16_t, 3); else LD4(f16_t, 4);
  }
#undef LD4
}

void lora_up(DType dt, const LoraUpArgs& a, int N, int max_len, hipStream_t s) {
  // tall blocks amortise the U staging; shrink them until the grid fills the chip (>= 4 per CU)
  int col_blocks = 0;
  for (int m = 0; m < a.n; ++m) col_blocks += ceil_div(a.len[m], 128);
  int rows = 256;
  while (rows > 64 && (long)ceil_div(N, rows) * col_blocks < 1024) rows /= 2;
  dim3 grid(ceil_div(N, rows), ceil_div(max_len, 128), a.n);
  if (dt == DType::BF16) hipLaunchKernelGGL(lora_up_k<bf16_t>, grid, dim3(256), 0, s, a, rows, N);
  else hipLaunchKernelGGL(lora_up_k<f16_t>, grid, dim3(256), 0, s, a, rows, N);
}

int lora_wgrad_splits(int blocks, int N) {
  // aim for >= 2 blocks per CU; every split keeps at least 4 chunks of 64 tokens
  int S = ceil_div(512, blocks > 0 ? blocks : 1);
  const int max_s = ceil_div(N, 64) / 4;
  if (S > max_s) S = max_s;
  return S < 1 ? 1 : S;
}

void lora_wgrad(DType dt, DType odt, const LoraWgradArgs& a, int N, int S, hipStream_t s) {
  int blocks = 0;
  for (int m = 0; m < a.n; ++m) blocks += a.nblk[m];
  dim3 grid(blocks, S);
  BLLM_DISPATCH(odt, OT, {
    if (dt == DType::BF16) hipLaunchKernelGGL((lora_wgrad_k<bf16_t, OT>), grid, dim3(256), 0, s, a, N);
    else hipLaunchKernelGGL((lora_wgrad_k<f16_t, OT>), grid, dim3(256), 0, s, a, N);
    if (S > 1) {
      const long total = a.part_ld;
      const int g = (int)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
      hipLaunchKernelGGL(lora_reduce_k<OT>, dim3(g), dim3(256), 0, s, a, S, total);
    }
  });
}

void lora_reduce(DType odt, const LoraWgradArgs& a, int S, hipStream_t s) {
  BLLM_DISPATCH(odt, OT, {
    const long total = a.part_ld;
    const int g = (int)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
    hipLaunchKernelGGL(lora_reduce_k<OT>, dim3(g), dim3(256), 0, s, a, S, total);
  });
}

int lora_head_bwd_splits(int R, int V, long ldl) {
  const int slabs = (V + LHB_SUB * LHB_NSUB - 1) / (LHB_SUB * LHB_NSUB);
  // one whole wave of resident workgroups (2 per CU: LDS-bound): a partial last wave of
  // workgroups leaves most CUs idle while it streams its row ranges (512 measured best of
  // 512 / 768 / 1,024 / 1,536 / 2,048, profiles/r5/lora_head/)
  int S = 512 / slabs;
  const int max_s = (R + 4 * LHB_ROWS - 1) / (4 * LHB_ROWS);  // >= 4 chunks per row range
  if (S > max_s) S = max_s;
  if (S < 1) S = 1;
  // the kernel's buffer offsets are 32-bit: a row range (plus the prefetch overrun) stays < 2 GB
  while (((long)(R + S - 1) / S + 4 * LHB_ROWS) * ldl * 2 >= 0x7ff00000L) ++S;
  return S;
}
void lora_head_bwd(DType dt, const void* dl, long ldl, const void* st, long ldst, const void* B, long ldb,
                   float* gpart, float* upart, void* u, int R, int V, int S, hipStream_t s) {
  const int slabs = (V + LHB_SUB * LHB_NSUB - 1) / (LHB_SUB * LHB_NSUB);
  const int rows_per = ((R + S - 1) / S + LHB_ROWS - 1) / LHB_ROWS * LHB_ROWS;
  const dim3 grid(slabs, S);
  const long n = (long)R * 16;
  // prefetch depth 4 (measured against 1 and 2, profiles/r5/lora_head/sweep*.txt)
  if (dt == DType::BF16) {
    hipLaunchKernelGGL((lora_head_bwd_k<bf16_t, 4>), grid, dim3(256), 0, s, (const bf16_t*)dl, ldl,
                       (const bf16_t*)st, ldst, (const bf16_t*)B, ldb, gpart, upart, R, V, rows_per);
    hipLaunchKernelGGL(lhb_usum_k<bf16_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, upart, (bf16_t*)u, n,
                       slabs);
  } else {
    hipLaunchKernelGGL((lora_head_bwd_k<f16_t, 4>), grid, dim3(256), 0, s, (const f16_t*)dl, ldl,
                       (const f16_t*)st, ldst, (const f16_t*)B, ldb, gpart, upart, R, V, rows_per);
    hipLaunchKernelGGL(lhb_usum_k<f16_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, upart, (f16_t*)u, n,
                       slabs);
  }
}

void lora_pack_t(DType dt, const LoraPackArgs& a, int K, int max_r, hipStream_t s) {
  dim3 grid(ceil_div((long)K * max_r, 256) < 256 ? ceil_div((long)K * max_r, 256) : 256, a.n);
  if (dt == DType::BF16) hipLaunchKernelGGL(lora_pack_t_k<bf16_t>, grid, dim3(256), 0, s, a, K);
  else hipLaunchKernelGGL(lora_pack_t_k<f16_t>, grid, dim3(256), 0, s, a, K);
}

}  // namespace bllm
