// Host launch API of the kernel library (raw pointers + hipStream_t; no torch types so the
// .hip translation units compile without PyTorch headers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "common.h"

namespace bllm {

// norms.hip
int norm_bwd_num_wg(int N, int d);
int norm_max_dim(DType dt);
void rmsnorm_fwd(DType dt, const void* x, const void* w, void* y, float* rstd, int N, int d, float eps, long ldy,
                 hipStream_t s);
void layernorm_fwd(DType dt, const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int N,
                   int d, float eps, hipStream_t s);
// dW / dB land in `dw` / `db` of dtype `odt` (written, or added when `accumulate`)
void rmsnorm_bwd(DType dt, const void* dy, const void* x, const void* w, const float* rstd, const void* dx_acc,
                 void* dx, float* part, DType odt, void* dw, bool accumulate, int N, int d, int nwg, hipStream_t s);
void layernorm_bwd(DType dt, const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                   const void* dx_acc, void* dx, float* part_w, float* part_b, DType odt, void* dw, void* db,
                   bool accumulate, int N, int d, int nwg, hipStream_t s);
// x2 = x + dropout(a) (stored) and y = LayerNorm(x2) in one pass (GPT-2 attention residual + norm2)
void dropout_add_layernorm_fwd(DType dt, const void* x, const void* a, void* xs, const void* w, const void* b, void* y,
                               float* mean, float* rstd, int N, int d, float eps, float p, uint64_t seed,
                               uint64_t offset, hipStream_t s);
void col_reduce(const float* part, DType odt, void* out, int P, int d, bool accumulate, hipStream_t s);

// elementwise.hip
// out[C, R] = in[R, C]^T, 16-bit elements, R % 8 == 0 and C % 8 == 0
void transpose16(const void* in, void* out, long R, long C, hipStream_t s);
void swiglu_fwd(DType dt, const void* gu, void* act, long N, int F, long lda, hipStream_t s);
// SwiGLU backward with dact = base + scale . u P formed on the fly (down-projection LoRA dX)
bool swiglu_bwd_lr_ok(int r, int F);
// swiglu_bwd_lr plus the gate / up dB and down dA^T reductions over the same rows: fp32 partials
// part [S][3][16][F] (sum them with lora_reduce); u = dy B^T of the down LoRA, st = s t of gate|up
bool swiglu_bwd_lr_wgrad_ok(int r, int F);
int swiglu_bwd_lr_wgrad_splits(long N, int F);
void swiglu_bwd_lr_wgrad(DType dt, const void* gu, const void* base, long ldb, const void* u, long ldu, const void* P,
                         const void* st, long ldst, float scale, void* dgu, float* part, long N, int F, int S,
                         hipStream_t s);
void swiglu_bwd_lr(DType dt, const void* gu, const void* base, long ldb, const void* u, long ldu, const void* P, int r,
                   float scale, void* dgu, long N, int F, hipStream_t s);
// act (nullable, may alias dact): also write silu(g) * u there -- the activation-checkpoint
// recompute then needs no separate SwiGLU forward pass for the down projection's dW
void swiglu_bwd(DType dt, const void* gu, const void* dact, void* dgu, void* act, long N, int F, hipStream_t s);
void gelu_fwd(DType dt, const void* f, void* g, long n, hipStream_t s);
void gelu_bwd(DType dt, const void* f, const void* dg, void* df, long n, hipStream_t s);
void dropout_add(DType dt, const void* x, const void* a, void* out, long n, float p, uint64_t seed, uint64_t offset,
                 hipStream_t s);
void rope(DType dt, void* qkv, const float* cosT, const float* sinT, long N, int T, int H, int G, int hd,
          bool inverse, int pos_offset, hipStream_t s, const int* pos_dev = nullptr);

// attention (attn.hip dispatch; attn_mfma.hip / attn_bwd_mfma.hip / attn_f32.hip / attn_naive.hip)
// keep_mask (dropout > 0, bf16/fp16 MFMA kernels only, else nullptr): the forward writes the
// attention-dropout keep bits, uint32 words [B*H][ceil(T/32)][T] (bit j of word (kw, q) = key
// 32kw + j), the backward kernels read them instead of re-hashing every (q, key).  Words of
// tiles above the causal diagonal are never written or read.
bool attn_supported_head_dim(int hd);
bool attn_keep_mask_ok(DType dt, int hd);
void attn_fwd(DType dt, const void* qkv, void* o, float* lse, int B, int T, int H, int G, int hd, bool causal,
              float p, uint64_t seed, uint64_t offset, uint32_t* keep_mask, hipStream_t s);
void attn_bwd(DType dt, const void* qkv, const void* o, const float* lse, const void* dout, void* dqkv, float* delta,
              float* dq_acc, float* dkv_part, int B, int T, int H, int G, int hd, bool causal, float p, uint64_t seed,
              uint64_t offset, const uint32_t* keep_mask, const float* rcos, const float* rsin, hipStream_t s);
// GEMM tile -> workgroup placement (map 0 = XCD-contiguous M-bands, 1 = plain order, 2 = N-bands)
// and group depth (<= 0: default) of the dW kernel and of the forward-layout kernel
void set_wgrad_tile_map(int map, int group_m);
void set_gemm_nt_tile_map(int map, int group_m);
bool attn_mfma_head_dim(int hd);
void attn_fwd_naive(DType dt, const void* qkv, void* o, float* lse, int B, int T, int H, int G, int hd, bool causal,
                    float p, uint64_t seed, uint64_t offset, hipStream_t s);
void attn_bwd_naive(DType dt, const void* qkv, const void* o, const float* lse, const void* dout, void* dqkv,
                    float* delta, int B, int T, int H, int G, int hd, bool causal, float p, uint64_t seed,
                    uint64_t offset, hipStream_t s);

// attn_f32.hip: fp32 flash attention on v_mfma_f32_32x32x2_f32 (head dims 64 / 128)
bool attn_f32_head_dim(int hd);
void attn_fwd_f32(const float* qkv, float* o, float* lse, int B, int T, int H, int G, int hd, bool causal, float p,
                  uint64_t seed, uint64_t offset, hipStream_t s);
void attn_bwd_f32(const float* qkv, const float* o, const float* lse, const float* dout, float* dqkv, float* delta,
                  int B, int T, int H, int G, int hd, bool causal, float p, uint64_t seed, uint64_t offset,
                  hipStream_t s);

// whether the dK/dV pass needs the fp32 per-head partial buffer (GQA without the fused-head variant)
bool attn_bwd_kv_partials(int B, int T, int H, int G);

void attn_delta(DType dt, const void* o, const void* dout, float* delta, int B, int T, int H, int hd,
                hipStream_t s);

// elementwise.hip — bias gradient (column sums), part must hold colsum_bands(N, F) * F floats
int colsum_bands(int N, int F);
// op 0: out = dropout_bwd(src), op 1: out = src * gelu'(aux); db (+)= out.sum(0) from the same pass
// (part == nullptr: no sums); op 1 with act: also act = gelu(aux) (may alias src)
void bwd_bias_grad(DType dt, DType odt, int op, const void* src, const void* aux, void* out, float* part, void* db,
                   int N, int F, bool accumulate, float p, uint64_t seed, uint64_t offset, void* act, hipStream_t s);
void bias_grad(DType dt, DType odt, const void* dy, float* part, void* out, int N, int F, bool accumulate,
               hipStream_t s);

// elementwise.hip — out[e] (+)= sum_s part[s][e] (n % 8 == 0)
void sum_partials_into(DType pdt, DType odt, const void* part, void* out, long n, int S, bool accumulate,
                       hipStream_t s);

// attn_decode.hip — single-query attention over a [B, G, Tmax, hd] KV cache
int attn_decode_max_len();
// graph-replayable decode step: q / new k / new v read from the packed qkv rows [B, (H+2G)*hd],
// the position from device memory (*pos), new k/v appended to the caches at *pos, attention
// over the pos + 1 keys -> out [B, H*hd]
void attn_decode_append(DType dt, const void* qkv, void* kc, void* vc, void* out, const int* pos, int B, int H,
                        int G, int hd, int Tmax, hipStream_t s);
void attn_decode(DType dt, const void* q, const void* kc, const void* vc, void* out, int B, int H, int G, int hd,
                 int Tmax, int L, hipStream_t s);

// loss.hip
void ce_fwd(DType dt, const void* logits, const int64_t* tgt, float* loss, float* lse, long N, long V, long ld,
            long ignore_index, hipStream_t s);
void ce_bwd(DType dt, void* logits, const int64_t* tgt, const float* lse, const float* scale, long N, long V, long ld,
            long ignore_index, hipStream_t s);

// embedding.hip
// kernel debug mode (common.h BLLM_DASSERT): first failed check code of each TU, reset on read
unsigned int debug_take_embedding();
unsigned int debug_take_loss();
unsigned int debug_take_attn_decode();
unsigned int debug_take_elementwise();
void embedding_fwd(DType dt, const int64_t* idx, const void* wte, const void* wpe, void* out, long N, int d, int T,
                   float p, uint64_t seed, uint64_t offset, long vocab, hipStream_t s);
long embedding_bwd_part_floats(long N, int d);  // fp32 scratch the token backward needs
void embedding_bwd_tok(DType dt, const int64_t* sorted, const int64_t* perm, const void* dx, void* grad, float* part,
                       long N, int d, bool accumulate, hipStream_t s);
void embedding_bwd_pos(DType dt, const void* dx, void* grad, int B, int T, int d, bool accumulate, hipStream_t s);

// lora.hip — see the file header for the operand conventions
constexpr int LORA_MAX = 8;
struct LoraDownArgs {  // chunk c: out[:, ocol_c : +16*nt_c] = x[:, c0_c : +len_c] . W_c^T
  const void* x; long ldx;
  void* out; long ldo;
  int R, zpad;                 // out columns [R, R + zpad) are written with zeros
  float scale;
  int n;
  int c0[LORA_MAX], len[LORA_MAX], ocol[LORA_MAX], nt[LORA_MAX];
  const void* w[LORA_MAX]; long ldw[LORA_MAX];
};
struct LoraUpArgs {  // member m: y[:, c0_m : +len_m] = base + bias + scale . t[:, toff_m : +r_m] . U_m
  void* y; long ldy;
  const void* base; long ldb;  // optional (may alias y)
  const void* bias;            // optional, indexed by absolute column
  const void* t; long ldt;
  float scale;
  int n;
  int c0[LORA_MAX], len[LORA_MAX], toff[LORA_MAX], r[LORA_MAX];
  const void* u[LORA_MAX]; long su_j[LORA_MAX], su_c[LORA_MAX];
};
struct LoraWgradArgs {  // member m: G_m[a*sa + b*sb] (+)= scale . sum_n p[n][pa_m + a] q[n][qb_m + b]
  const void* p; long ldp;
  const void* q; long ldq;
  float scale;
  bool accumulate;
  int n;
  int pa[LORA_MAX], qb[LORA_MAX], r[LORA_MAX], len[LORA_MAX], nblk[LORA_MAX];
  long sa[LORA_MAX], sb[LORA_MAX];
  void* gt[LORA_MAX][4];       // output of member m's 16-column tile t (element [0][0] of that tile)
  float* part; long part_ld; long part_off[LORA_MAX];  // S > 1: part[s][part_off_m + a * len_m + b]
};
struct LoraPackArgs {  // out[off_m + j][k] = a_m[k][j]
  void* out;
  int n;
  int off[LORA_MAX], r[LORA_MAX];
  const void* a[LORA_MAX];
};
struct LoraBlockArgs {  // dst[row * s_row + j * s_j] = B_m[j - off_m][row - c0_m] inside member m's block, else 0
  void* dst; long s_row, s_j;
  int rows, R;
  int n;
  int c0[LORA_MAX], len[LORA_MAX], off[LORA_MAX], r[LORA_MAX];
  const void* b[LORA_MAX]; long ldb[LORA_MAX];
};
void lora_down(DType dt, const LoraDownArgs& a, int N, hipStream_t s);
void lora_block(DType dt, const LoraBlockArgs& a, hipStream_t s);
void lora_up(DType dt, const LoraUpArgs& a, int N, int max_len, hipStream_t s);
int lora_wgrad_splits(int blocks, int N);
void lora_wgrad(DType dt, DType odt, const LoraWgradArgs& a, int N, int S, hipStream_t s);
// g_m (+)= sum_s part[s][part_off_m + a * len_m + b] (a.part, a.part_ld, a.part_off set; scale not applied)
void lora_reduce(DType odt, const LoraWgradArgs& a, int S, hipStream_t s);
// the LoRA head's u = dl B^T (written to u [R, 16] via partials per 1,024-column slab, upart
// [slabs][R][16]) and dB = st^T dl (partials per row range: gpart [S][16][V], summed by the caller
// with lora_reduce) in one pass over dl (V % 64 == 0, r = 16)
int lora_head_bwd_splits(int R, int V, long ldl);
void lora_head_bwd(DType dt, const void* dl, long ldl, const void* st, long ldst, const void* B, long ldb,
                   float* gpart, float* upart, void* u, int R, int V, int S, hipStream_t s);
void lora_pack_t(DType dt, const LoraPackArgs& a, int K, int max_r, hipStream_t s);

// gemm_wgrad.hip — C[M, N] (+)= A^T B with A [K, M], B [K, N] row-major (dW = dY^T X).
// S > 1: split s writes fp32 partial C + s * c_split (accumulate must be false).
bool wgrad_gemm_supported(int M, int N, int K, int S);
bool wgrad_tail_supported(int M, int N, int K, int full, int St);
// tiles [0, full) whole-K into c, the rest split St ways into compact fp32 partials (part) + a sum
void wgrad_gemm_tail(DType dt, DType odt, const void* a, long lda, const void* b, long ldb, void* c, long ldc, int M,
                     int N, int K, int full, int St, float* part, bool accumulate, hipStream_t s);
void wgrad_gemm(DType dt, DType odt, const void* a, long lda, const void* b, long ldb, void* c, long ldc,
                long c_split, int M, int N, int K, int S, bool accumulate, hipStream_t s);
// same kernel with a K-contiguous A: C[M, N] (+)= A[M, K] B[K, N] (dX = dY W)
bool gemm_nn_supported(int M, int N, int K);
void gemm_nn(DType dt, DType odt, const void* a, long lda, const void* b, long ldb, void* c, long ldc, int M, int N,
             int K, bool accumulate, hipStream_t s);

// gemm_nt.hip — persistent 4-wave forward-layout kernel with 64-deep K-tiles (full 128-B rows):
// C[M, N] (+)= A[M, K] B[N, K]^T; M, N multiples of 256, K of 128
bool gemm_nt2_supported(int M, int N, int K, long lda, long ldb);
void gemm_nt2(DType dt, DType odt, const void* a, long lda, const void* b, long ldb, void* c, long ldc, int M, int N,
              int K, bool accumulate, hipStream_t s);
// gate/up projection with the SwiGLU forward in the epilogue: gu[M, 2F] = a . [Wg; Wu]^T and
// act[M, F] = silu(gu[:, :F]) * gu[:, F:] (bitwise the separate swiglu_fwd)
bool gemm_nt_swiglu_supported(int M, int F, int K, long lda, long ldb, long ldgu);
// qkv [M, N] = a [M, K] . w [N, K]^T with RoPE applied to columns < nrot (head dim 128) at
// position row % Tq in the epilogue of the persistent 4-wave kernel (csrc/gemm_nt.hip)
bool gemm_nt_rope_supported(int M, int N, int K, long lda, long ldb, long ldc, int hd);
// GPT-2 c_fc with bias + exact GELU in the epilogue: f = a . w^T + bias, g = gelu(f) (both [M, N])
bool gemm_nt_bias_gelu_supported(int M, int N, int K, long lda, long ldb, long ldc);
void gemm_nt_bias_gelu(DType dt, const void* a, long lda, const void* w, long ldw, const void* bias, void* f, void* g,
                       long ldc, int M, int N, int K, hipStream_t s);
void gemm_nt_rope(DType dt, const void* a, long lda, const void* w, long ldw, void* c, long ldc, int M, int N, int K,
                  const float* cosT, const float* sinT, int Tq, int nrot, hipStream_t s);
void gemm_nt_swiglu(DType dt, const void* a, long lda, const void* w, long ldw, void* gu, long ldgu, void* act, int M,
                    int F, int K, hipStream_t s);

// optim.hip
void adamw_step(DType pdt, DType gdt, void* param, float* master, const void* grad, float* m, float* v, long n,
                float lr, float b1, float b2, float eps, float wd, int step, const float* gscale, hipStream_t s);
int sqsum_slots(long n);
void sqsum_partial(DType dt, const void* x, long n, float* part, int slots, hipStream_t s);
void sum_partials(const float* part, int n, float* out, hipStream_t s);

}  // namespace bllm
