/*
 * lightglue_glue.h — gfx950 kernels for the LightGlue matcher built around MHAHeadDim64
 * (SURVEY.md section 8(f) ranks 3/4). Not part of the reference plugin's surface: these
 * replace chains of small framework ops around the attention call in
 * lightglue_pytorch_no_plugin/lightglue.py (one launch each instead of 3-8).
 *
 * Layouts are row-major and contiguous. dtype: MHA_HD64_DT_FLOAT (0) or MHA_HD64_DT_HALF (1)
 * for every tensor argument of a call (statistics and softmax math in fp32). All calls are
 * asynchronous on `stream` and return 0 or a nonzero status (message: mha_hd64_last_error()).
 *
 * Image pairs: the row-major side of the split/merge calls holds `pairs` image pairs stacked
 * pair-major — pair p's n0 rows of image 0, then its n1 rows of image 1 — so "[n0+n1, ...]"
 * below reads [pairs*(n0+n1), ...], and each per-image head-major tensor "[heads, ni, 64]" reads
 * [pairs, heads, ni, 64] (the batch dimension of the attention calls). pairs = 1: one pair.
 *
 * ABI version 2 (round 4): `pairs` inserted after n1 in the split / merge / fused-projection calls
 * and `batch` in the dual log-softmax and its workspace query. A host built against an older
 * header links against the same symbol names and would pass shifted arguments: check
 * lg_glue_abi_version() == LG_GLUE_ABI_VERSION once at load.
 * ABI version 3 (round 6): lg_linear_cat_ffn takes the packed weight stream of its one-launch form
 * (w_packed, after b2; lg_ffn_pack). ABI version 4: lg_ffn_pack writes two layouts (the 16-row
 * kernel's after the 32-row kernel's; lg_ffn_packed_bytes doubled).
 */
#ifndef LIGHTGLUE_GLUE_H_
#define LIGHTGLUE_GLUE_H_

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LG_GLUE_ABI_VERSION 4
/* The ABI version of the argument lists below that this library implements. */
int32_t lg_glue_abi_version(void);

/* SelfBlock q/k/v (lightglue.py:111-119, rotary :124-134): qkv [n0+n1, heads*64*3] is the Wqkv
 * output with channel (h*64 + d)*3 + j; cos/sin [n0+n1, 64] the positional encoding (pairs
 * repeated, lightglue.py:44-52). Writes q/k (rotated) and v of image i as [heads, ni, 64]. */
int32_t lg_qkv_rotary_split(int32_t dtype, const void* qkv, const void* cos, const void* sin, int32_t heads,
                            int32_t n0, int32_t n1, int32_t pairs, void* q0, void* k0, void* v0, void* q1, void* k1,
                            void* v1, hipStream_t stream);

/* CrossBlock heads (lightglue.py:158-166): a, b [n0+n1, heads*64] -> a0, b0 [heads, n0, 64],
 * a1, b1 [heads, n1, 64]. */
int32_t lg_split_heads2(int32_t dtype, const void* a, const void* b, int32_t heads, int32_t n0, int32_t n1,
                        int32_t pairs, void* a0, void* a1, void* b0, void* b1, hipStream_t stream);

/* The same with row stride `ld` elements for a and b (column views of one wider projection, e.g.
 * the cross block's to_qk | to_v computed as one GEMM: a = qkv, b = qkv + heads*64, ld = 2*heads*64);
 * a and b 16-byte aligned. */
int32_t lg_split_heads2_ld(int32_t dtype, const void* a, const void* b, int32_t ld, int32_t heads, int32_t n0,
                           int32_t n1, int32_t pairs, void* a0, void* a1, void* b0, void* b1, hipStream_t stream);

/* Attention outputs back to rows (lightglue.py:118-120, 163-170): x0 [heads, n0, 64],
 * x1 [heads, n1, 64] -> out [n0+n1, heads*64]. */
int32_t lg_merge_heads(int32_t dtype, const void* x0, const void* x1, int32_t heads, int32_t n0, int32_t n1,
                       int32_t pairs, void* out, hipStream_t stream);

/* The FFN input of both blocks (lightglue.py:104, 181: cat([x, message], -1)) with the message
 * projection folded into the FFN's first weight: out [n0+n1, 2*heads*64] = [x | merge(x0, x1)],
 * x [n0+n1, heads*64]. One pass instead of merge_heads + a concatenation copy. */
int32_t lg_merge_heads_cat(int32_t dtype, const void* x, const void* x0, const void* x1, int32_t heads, int32_t n0,
                           int32_t n1, int32_t pairs, void* out, hipStream_t stream);

/* FFN middle (lightglue.py:101-106): y = GELU(LayerNorm(x) * gamma + beta), exact (erf) GELU,
 * x, y [rows, dim], dim a multiple of 64 and <= 1024; y == x (in place) is allowed: each row is read
 * whole before any of it is written. */
int32_t lg_layernorm_gelu(int32_t dtype, const void* x, const void* gamma, const void* beta, int32_t rows,
                          int32_t dim, float eps, void* y, hipStream_t stream);

/* ---- projections with their neighbours fused (fp16 only; csrc/lightglue_linear.hip) ----
 * W [n, k] row-major (nn.Linear layout), bias [n]; k in {256, 512}; n a multiple of 64; rows m
 * any. A/W/x/ctx 16-byte aligned, bias/out/res/cos/sin 8-byte aligned.
 * lg_linear:            out [m, n] = A [m, k] · Wᵀ + bias (+ res [m, n] when res != NULL). */
int32_t lg_linear(const void* a, const void* w, const void* bias, const void* res, int32_t m, int32_t n, int32_t k,
                  void* out, hipStream_t stream);
/* lg_linear_cat:        out [n0+n1, n] = [x | merge_heads(ctx0, ctx1)] · Wᵀ + bias with x [n0+n1, heads*64],
 *                       ctx_i [heads, ni, 64] (k = 2*heads*64; the FFN input of lightglue.py:104/181). */
int32_t lg_linear_cat(const void* x, const void* ctx0, const void* ctx1, int32_t heads, int32_t n0, int32_t n1,
                      int32_t pairs, const void* w, const void* bias, int32_t n, void* out, hipStream_t stream);
/* lg_linear_cat_ln_gelu: the FFN's first half (lightglue.py:101-106) after lg_linear_cat:
 *                       out [n0+n1, 512] = GELU(LayerNorm(fp16([x | merge_heads(ctx0, ctx1)] · Wᵀ + bias)))
 *                       with the LayerNorm's gamma, beta [512] and eps (exact-erf GELU). One launch
 *                       (tiles owning whole rows: 64-row tiles from m >= 16,384, 128-row tiles from
 *                       m >= 32,768; heads * 128 = 512, 16-B aligned bias / gamma / beta / out), else
 *                       lg_linear_cat then lg_layernorm_gelu in place; see lg_linear_set_ln_fused. */
int32_t lg_linear_cat_ln_gelu(const void* x, const void* ctx0, const void* ctx1, int32_t heads, int32_t n0, int32_t n1,
                              int32_t pairs, const void* w, const void* bias, const void* gamma, const void* beta,
                              float eps, void* out, hipStream_t stream);
/* lg_linear_cat_ffn:    the whole FFN with the block's residual (lightglue.py:101-106, 150-151 / 174-175):
 *                       out [n0+n1, d] = x + fp16(W2 · GELU(LayerNorm(W1 · [x | merge_heads(ctx0, ctx1)] + b1)) + b2)
 *                       with d = heads*64 = 256, W1 [2d, 2d], W2 [d, 2d]. With w_packed (W1 and W2 as
 *                       lg_ffn_pack lays them out): ONE launch, whole rows per workgroup (16 rows up to
 *                       4,096 rows, ffn_rows16_kernel; 32 up to 8,192 and 64 beyond, ffn_rows_kernel; each
 *                       wave streams its own weight fragments into registers, the GELU output stays in
 *                       LDS; within 2 fp16 ulps of the two calls).
 *                       With w_packed NULL: lg_linear_cat_ln_gelu into h [m, 2d] then lg_linear(h, W2, b2,
 *                       res = x). h must hold m*2d fp16 either way (unused by the one-launch form); out
 *                       must not alias x (16-B aligned pointers). */
int32_t lg_linear_cat_ffn(const void* x, const void* ctx0, const void* ctx1, int32_t heads, int32_t n0, int32_t n1,
                          int32_t pairs, const void* w1, const void* b1, const void* gamma, const void* beta, float eps,
                          const void* w2, const void* b2, const void* w_packed, void* h, void* out, hipStream_t stream);
/* lg_ffn_pack:          W1 [2d, 2d] and W2 [d, 2d] (nn.Linear layout, fp16, d = heads*64 = 256), and for
 *                       lg_linear_cat_ffn_proj a W3 [n3, d] (n3 = 512 or 768; 0: none), re-laid as the
 *                       one-launch FFN reads them, twice. The 32-row kernel's layout: 8 wave streams of
 *                       (96 + n3/16) KiB, stream w = W1 rows 64w..64w+63 then W2 rows 32w..32w+31 then W3
 *                       rows (n3/8)w.., in 1-KiB pieces i (W1: step j, block b at i = 2j + b; W2: step j at
 *                       i = 64 + j; W3: step j, block b at i = 96 + (n3/256) j + b) whose 16-B lane l holds
 *                       W[row0 + 32b + (l % 32)][16j + 8(l / 32) .. + 8]; then the 16-row kernel's: the same
 *                       rows per stream in 16-row blocks and k32 steps (W1: i = 4j + b, W2: i = 64 + 2j + b,
 *                       W3: i = 96 + (n3/128) j + b), lane l = W[row0 + 16b + (l % 16)][32j + 8(l / 16) .. + 8]
 *                       — every load of either kernel one contiguous KiB. lg_ffn_packed_bytes(heads, n3):
 *                       the size of both (1,572,864 B for n3 = 0; 0 if heads != 4 or n3 is not 0 / 512 /
 *                       768).
 *                       Weights are static: pack once per weight update. lg_linear_cat_ffn takes an n3 = 0 pack. */
size_t lg_ffn_packed_bytes(int32_t heads, int32_t n3);
int32_t lg_ffn_pack(const void* w1, const void* w2, const void* w3, int32_t n3, int32_t heads, void* packed,
                    hipStream_t stream);
/* lg_linear_cat_ffn_proj: lg_linear_cat_ffn's one-launch form, then — in the same launch, on its output
 *                       out = x' still in LDS — the projection the next attention needs (the 32/64-row
 *                       forms bitwise the separate call's outputs; the 16-row form sums each k32 step in
 *                       one MFMA, within 1 fp16 ulp of them; round 6):
 *                         kind LG_PROJ_SPLIT2: W3 = [W_qk; W_v] [512, d], b3 [512] -> a0, a1, b0, b1 as
 *                                              lg_linear_split2 (outs3[0..3]);
 *                         kind LG_PROJ_QKV:    W3 = Wqkv permuted [768, d], b3 [768], cos / sin [m, 64] ->
 *                                              q0, k0, v0, q1, k1, v1 as lg_linear_qkv_rotary (outs3[0..5]);
 *                         kind LG_PROJ_PLAIN:  W3 [512, d] (rows past n_store zero), b3 [512] -> outs3[0]
 *                                              [m, n_store] = x' · W3ᵀ + b3 (n_store <= 512, % 8 == 0).
 *                       w_packed = lg_ffn_pack(W1, W2, W3, 512 or 768); out [m, d] as lg_linear_cat_ffn
 *                       (all pointers 16-B aligned but b3 / cos / sin, 8-B). heads must be 4. */
#define LG_PROJ_SPLIT2 1
#define LG_PROJ_QKV 2
#define LG_PROJ_PLAIN 3
int32_t lg_linear_cat_ffn_proj(const void* x, const void* ctx0, const void* ctx1, int32_t heads, int32_t n0, int32_t n1,
                               int32_t pairs, const void* b1, const void* gamma, const void* beta, float eps, const void* b2,
                               const void* w_packed, int32_t kind, const void* b3, const void* cosv, const void* sinv,
                               int32_t n_store, void* const* outs3, void* out, hipStream_t stream);
/* lg_linear_qkv_rotary: SelfBlock projection (lightglue.py:111-134) with W's rows and the bias in
 *                       [q|k|v][head][dim] order (row j*heads*64 + h*64 + d = Wqkv row (h*64+d)*3 + j):
 *                       rotary (cos/sin [n0+n1, 64]) on q and k in fp16 arithmetic, as the reference's
 *                       fp16 model rounds t * cos + rotate_half(t) * sin (each product and the sum),
 *                       per-image head-major outputs. */
int32_t lg_linear_qkv_rotary(const void* x, const void* w_perm, const void* b_perm, const void* cos, const void* sin,
                             int32_t heads, int32_t n0, int32_t n1, int32_t pairs, int32_t k, void* q0, void* k0,
                             void* v0, void* q1, void* k1, void* v1, hipStream_t stream);
/* lg_linear_split2:     CrossBlock to_qk | to_v as one projection (W = [W_qk; W_v], lightglue.py:158-166):
 *                       per-image head-major a (= qk) and b (= v). */
int32_t lg_linear_split2(const void* x, const void* w, const void* bias, int32_t heads, int32_t n0, int32_t n1,
                         int32_t pairs, int32_t k, void* a0, void* a1, void* b0, void* b1, hipStream_t stream);

/* sigmoid_log_double_softmax (lightglue.py:197-205), fp32: scores[i][j] = 2 sim[i][j]
 * - logsumexp_j' sim[i][j'] - logsumexp_i' sim[i'][j] + logsigmoid(z0[i]) + logsigmoid(z1[j]).
 * sim, scores [batch, m, n]; z0 [batch, m], z1 [batch, n] (batch image pairs, one launch);
 * workspace >= lg_log_double_softmax_workspace(m, n, batch) bytes. */
size_t lg_log_double_softmax_workspace(int32_t m, int32_t n, int32_t batch);
int32_t lg_log_double_softmax(const float* sim, const float* z0, const float* z1, int32_t m, int32_t n, int32_t batch,
                              float* scores, void* workspace, hipStream_t stream);

/* The same on the fp16 model's outputs (round 5): sim [batch, m, n] fp16 (16-B aligned, n % 8 == 0,
 * n <= 2048) read directly, the matchability logits fp16 and strided — z0 of pair p, row i at
 * z0[p * z_pair_stride + i * z_row_stride], z1 of pair p, column j at z1[p * z_pair_stride + j *
 * z_row_stride] (one channel of the final projection's output) — scores fp32 (16-B aligned). Two
 * launches; workspace >= lg_log_double_softmax_f16_workspace(m, n, batch) bytes. */
size_t lg_log_double_softmax_f16_workspace(int32_t m, int32_t n, int32_t batch);
int32_t lg_log_double_softmax_f16(const void* sim, const void* z0, const void* z1, int64_t z_pair_stride,
                                  int64_t z_row_stride, int32_t m, int32_t n, int32_t batch, float* scores,
                                  void* workspace, hipStream_t stream);

/* The fp16 assignment head in two launches (round 6): v [batch][m + n][ld] fp16 is the final
 * projection of both images' rows (image 0's m rows, then image 1's n; pairs pair_stride elements
 * apart), channels 0..255 the scaled descriptors m0 / m1 (final_proj(d) / d^0.25) and channel zc
 * (>= 256) the matchability logit. scores [batch, m, n] fp32 = log_softmax(sim, 2) + log_softmax(sim, 1)
 * + logsig(z0) + logsig(z1)ᵀ with sim = m0 · m1ᵀ rounded to fp16 (lightglue.py:208-233): the similarity
 * by MFMA with each row's and column's (max, sum of exponentials) over shares of the other image (a
 * workgroup owns 32 rows of one image), then the combine, which closes its rows' and columns'
 * logsumexps from those partials.
 * m, n <= 2048, n % 8 == 0, ld % 8 == 0; v, scores, workspace 16-B aligned; workspace >=
 * lg_assign_scores_workspace(m, n, batch) bytes (its first batch * m * n * 2 bytes: sim, fp16). */
size_t lg_assign_scores_workspace(int32_t m, int32_t n, int32_t batch);
int32_t lg_assign_scores(const void* v, int64_t pair_stride, int32_t ld, int32_t zc, int32_t m, int32_t n, int32_t batch,
                         float* scores, void* workspace, hipStream_t stream);

/* The fp16 forward's inputs (lightglue.py:329-337 and FourierPositionalEncoding :32-52), round 5:
 * x [pairs * (n0 + n1), dim] pair-major from desc0 [pairs, n0, dim] and desc1 [pairs, n1, dim]
 * (dim = 256, 16-B aligned), and the rotary tables cos, sin [pairs * (n0 + n1), 64] from kpts0
 * [pairs, n0, 2], kpts1 [pairs, n1, 2] and Wr [32, 2] (all fp16): proj = Wr · kpt rounded to fp16,
 * cos / sin of it rounded to fp16, each value repeated for the two members of a rotary pair. */
int32_t lg_pair_inputs(const void* desc0, const void* desc1, const void* kpts0, const void* kpts1, const void* wr,
                       int32_t n0, int32_t n1, int32_t pairs, int32_t dim, void* x, void* cosv, void* sinv,
                       hipStream_t stream);

/* Test and benchmark hook: the projections' tile forms for launches of many rows (several image
 * pairs per forward): 0 the 64 x 64 form only, 4 the 128 x 128 form on 4 waves (two workgroups per
 * CU; the by-size choice from 128 of its tiles and 8,192 rows on), -1 (the default) chosen by size;
 * 1 the 256 x 128 form and 2 the 256 x 256 form (plain bias outputs; else 1) where n allows — in A/B
 * builds only (-DLG_LINEAR_AB_FORMS=1, tools/build_linear_variant.sh); the shipped library runs form 4
 * for them, as for 3 and 5 (round 5's A/B forms, removed); values outside -1..5 are clamped. The environment variable LG_LINEAR_WIDE sets the initial mode the same way. Every form
 * gives the same bits. Returns the previous mode. */
int32_t lg_linear_set_wide(int32_t mode);

/* Test and benchmark hook for lg_linear_cat_ln_gelu's forms: 1 (the default) one launch from a full
 * round of its tiles on, 0 always two launches, 2 always one launch (A/B). The forms agree within fp16
 * rounding, not in every bit (the one-launch variance is two-pass). Returns the previous setting. */
int32_t lg_linear_set_ln_fused(int32_t on);
/* Test and benchmark hook for lg_linear_cat_ffn's (and lg_linear_cat_ffn_proj's) forms: 1 (the
 * default) the one-launch form when w_packed is given, its kernel by size (16-row tiles up to 4,096
 * rows, then 32-row up to 8,192, then 64-row); 2 the 32/64-row kernel at every size, 3 the 16-row
 * kernel at every size (A/B); 0 always the two calls (lg_linear_cat_ffn; lg_linear_cat_ffn_proj has
 * only the one-launch form and takes 0 as 1). Values outside 0..3 select 1. Returns the previous
 * setting. */
int32_t lg_linear_set_ffn_fused(int32_t mode);

#ifdef __cplusplus
}
#endif

#endif /* LIGHTGLUE_GLUE_H_ */
