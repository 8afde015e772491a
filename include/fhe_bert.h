/*
 * fhe_bert.h — C ABI of the embedding stage's encoder in libfheicp.so
 * (SURVEY.md §8 f4): a BERT forward pass on gfx950 (MFMA GEMMs, a fused
 * flash-style attention kernel, fp32 LayerNorm / residual stream).
 *
 * Boundary. The reference embeds documents with
 * BertEmbedder.get_embedding / get_embeddings_batch
 * (bert_embeddings.py:53-101, :103-158): tokenizer -> transformers
 * AutoModel('bert-base-uncased') forward (:45, :136) -> last_hidden_state ->
 * mean / cls / max pooling (:140-149) -> float32 numpy. Everything from the
 * token ids to the pooled embedding is replaced by fhe_bert_forward; the
 * tokenizer stays on the host (fhe-icp_amd/bert_embeddings.py mirrors the
 * reference class). Weights are the transformers BertModel state_dict
 * (float32 host arrays, torch layout [out][in]), loaded once.
 *
 * Numerics (fhe_bert_set_precision):
 *  - FHE_BERT_F32 (default): the reference's arithmetic. Every GEMM and both
 *    attention products are f32 x f32 on v_mfma_f32_32x32x2_f32 (an exact f32
 *    fma chain per output), f32 bias / GELU (library erff) / residual /
 *    LayerNorm / softmax / pooling: torch's fp32 forward in another summation
 *    order (tests/test_gpu_bert.py: hidden-state relative RMS <= 1e-5).
 *  - FHE_BERT_BF16 (opt-in): GEMM and attention operands in bf16 (weights
 *    rounded once at load, activations at each GEMM input), fp32
 *    accumulation; ~3x faster, agreeing with the fp32 reference only to the
 *    looser tolerance tests/test_gpu_bert.py states.
 * Neither is bit-equal to torch (real-weight parity is unpinned: the weights
 * are offline). A changed embedding can move a PCA feature across an input-
 * quantizer rounding boundary, so the mirrors tag what this encoder embedded
 * (DESIGN.md §7).
 *
 * Conventions as fhe_icp.h: 0 on success, negative FHE_E_* on failure,
 * fhe_bert_last_error for the message; d_* are device pointers; stream is a
 * hipStream_t as void*. One handle per device, calls externally serialised.
 */
#ifndef FHE_BERT_H
#define FHE_BERT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fhe_bert_config {
  int32_t vocab_size;          /* 30522 for bert-base-uncased */
  int32_t hidden_size;         /* 768; must be num_heads * 64 and a multiple of 64 */
  int32_t num_layers;          /* 12 */
  int32_t num_heads;           /* 12 (head dim 64) */
  int32_t intermediate_size;   /* 3072; a multiple of 64 */
  int32_t max_position;        /* 512 (also the longest sequence) */
  int32_t type_vocab_size;     /* 2 */
  float layer_norm_eps;        /* 1e-12 */
} fhe_bert_config;

typedef struct fhe_bert fhe_bert;

/* tensor ids of fhe_bert_set_tensor (HF BertModel state_dict names):
 * per model (layer = -1): embeddings.{word,position,token_type}_embeddings,
 * embeddings.LayerNorm.{weight,bias}; per layer l: attention.self.{query,
 * key,value}.{weight,bias}, attention.output.dense.{weight,bias},
 * attention.output.LayerNorm.{weight,bias}, intermediate.dense.{weight,
 * bias}, output.dense.{weight,bias}, output.LayerNorm.{weight,bias}. */
enum {
  FHE_BERT_WORD_EMB = 0, FHE_BERT_POS_EMB, FHE_BERT_TYPE_EMB, FHE_BERT_EMB_LN_W, FHE_BERT_EMB_LN_B,
  FHE_BERT_Q_W = 16, FHE_BERT_Q_B, FHE_BERT_K_W, FHE_BERT_K_B, FHE_BERT_V_W, FHE_BERT_V_B,
  FHE_BERT_AO_W, FHE_BERT_AO_B, FHE_BERT_AO_LN_W, FHE_BERT_AO_LN_B,
  FHE_BERT_I_W, FHE_BERT_I_B, FHE_BERT_O_W, FHE_BERT_O_B, FHE_BERT_O_LN_W, FHE_BERT_O_LN_B
};
/* pooling of fhe_bert_forward (bert_embeddings.py:140-149) */
enum { FHE_BERT_POOL_MEAN = 0, FHE_BERT_POOL_CLS = 1, FHE_BERT_POOL_MAX = 2, FHE_BERT_POOL_NONE = 3 };
/* arithmetic of the forward pass (see Numerics above) */
enum { FHE_BERT_F32 = 0, FHE_BERT_BF16 = 1 };

/* New handle on `device` (precision FHE_BERT_F32). */
int fhe_bert_create(const fhe_bert_config* cfg, int device, fhe_bert** out);
/* Select FHE_BERT_F32 or FHE_BERT_BF16; only before the first
 * fhe_bert_set_tensor (FHE_E_STATE after: the weights are stored in the
 * selected type). fhe_bert_get_precision returns the current one. */
int fhe_bert_set_precision(fhe_bert* h, int32_t precision);
int fhe_bert_get_precision(const fhe_bert* h);
void fhe_bert_destroy(fhe_bert* h);
const char* fhe_bert_last_error(const fhe_bert* h);
/* Copy one float32 host tensor (count elements, torch layout) to the device,
 * converting GEMM weights to bf16 under FHE_BERT_BF16; synchronous. */
int fhe_bert_set_tensor(fhe_bert* h, int32_t layer, int32_t which, const float* h_data, int64_t count);
/* 1 once every tensor of the config has been set */
int fhe_bert_ready(const fhe_bert* h);
/* Forward pass of B sequences of S tokens (row-major [B][S] int32 device
 * arrays: token ids, token type ids (NULL: all 0), attention mask 0/1; S <=
 * max_position; every row needs mask[b][0] = 1, as the tokenizer's [CLS]).
 * pooling MEAN / CLS / MAX writes d_out [B][hidden] float32 (mean over the
 * mask, row 0, max over all S positions, as bert_embeddings.py:140-149);
 * NONE writes last_hidden_state [B][S][hidden] float32. Workspace grows on
 * demand (B*S*(hidden*24 + intermediate*4) bytes under FHE_BERT_F32,
 * B*S*(hidden*18 + intermediate*2) under FHE_BERT_BF16). */
int fhe_bert_forward(fhe_bert* h, const int32_t* d_ids, const int32_t* d_type_ids, const int32_t* d_mask, int32_t B,
                     int32_t S, int32_t pooling, float* d_out, void* stream);
/* Measurement: with profiling on, fhe_bert_forward brackets its kernel
 * classes with hipEvents; kernel = "gemm", "attention" or "other"; returns
 * total ms, launches and the algorithmic FLOPs of those launches, then
 * resets them. */
int fhe_bert_profile_enable(fhe_bert* h, int enable);
int fhe_bert_profile_read(fhe_bert* h, const char* kernel, double* total_ms, int64_t* launches, double* flops);

#ifdef __cplusplus
}
#endif
#endif /* FHE_BERT_H */
