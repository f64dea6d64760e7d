// Attention dispatch: MFMA flash-attention kernels for the head dims they tile (bf16/fp16:
// attn_mfma.hip / attn_bwd_mfma.hip; fp32: attn_f32.hip), the scalar kernels (attn_naive.hip)
// otherwise.  No dtype materialises the [B,H,T,T] scores.
#include "api.h"

namespace bllm {

void attn_fwd_mfma(DType dt, const void* qkv, void* o, float* lse, int B, int T, int H, int G, int hd, bool causal,
                   float p, uint64_t seed, uint64_t offset, uint32_t* keep_mask, hipStream_t s);
void attn_bwd_mfma(DType dt, const void* qkv, const void* o, const float* lse, const void* dout, void* dqkv,
                   float* delta, float* dq_acc, float* dkv_part, int B, int T, int H, int G, int hd, bool causal,
                   float p, uint64_t seed, uint64_t offset, const uint32_t* keep_mask, const float* rcos,
                   const float* rsin, hipStream_t s);

bool attn_supported_head_dim(int hd) { return hd > 0 && hd <= 256; }
bool attn_keep_mask_ok(DType dt, int hd) { return dt != DType::F32 && attn_mfma_head_dim(hd); }

void attn_fwd(DType dt, const void* qkv, void* o, float* lse, int B, int T, int H, int G, int hd, bool causal,
              float p, uint64_t seed, uint64_t offset, uint32_t* keep_mask, hipStream_t s) {
  if (dt == DType::F32 && attn_f32_head_dim(hd))
    attn_fwd_f32((const float*)qkv, (float*)o, lse, B, T, H, G, hd, causal, p, seed, offset, s);
  else if (dt != DType::F32 && attn_mfma_head_dim(hd))
    attn_fwd_mfma(dt, qkv, o, lse, B, T, H, G, hd, causal, p, seed, offset, p > 0.f ? keep_mask : nullptr, s);
  else
    attn_fwd_naive(dt, qkv, o, lse, B, T, H, G, hd, causal, p, seed, offset, s);
}

void attn_bwd(DType dt, const void* qkv, const void* o, const float* lse, const void* dout, void* dqkv, float* delta,
              float* dq_acc, float* dkv_part, int B, int T, int H, int G, int hd, bool causal, float p, uint64_t seed,
              uint64_t offset, const uint32_t* keep_mask, const float* rcos, const float* rsin, hipStream_t s) {
  if (dt != DType::F32 && attn_mfma_head_dim(hd)) {  // inverse RoPE fused into the epilogues
    attn_bwd_mfma(dt, qkv, o, lse, dout, dqkv, delta, dq_acc, dkv_part, B, T, H, G, hd, causal, p, seed, offset,
                  p > 0.f ? keep_mask : nullptr, rcos, rsin, s);
    return;
  }
  if (dt == DType::F32 && attn_f32_head_dim(hd))
    attn_bwd_f32((const float*)qkv, (const float*)o, lse, (const float*)dout, (float*)dqkv, delta, B, T, H, G, hd,
                 causal, p, seed, offset, s);
  else
    attn_bwd_naive(dt, qkv, o, lse, dout, dqkv, delta, B, T, H, G, hd, causal, p, seed, offset, s);
  if (rcos) rope(dt, dqkv, rcos, rsin, (long)B * T, T, H, G, hd, /*inverse=*/true, 0, s, nullptr);
}

}  // namespace bllm
