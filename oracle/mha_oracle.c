/*
 * mha_oracle.c — CPU restatement of the reference's MHAHeadDim64 attention.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker. The product
 * path (lightglue_amd + lib/libmha_hd64.so) never calls it.
 *
 * Parity anchor: outputs of the reference's own PyTorch attention
 * (lightglue_pytorch_no_plugin/lightglue.py:75-85), imported in the build
 * container and committed as tests/golden/attn_<case>.npz by tests/golden/make_golden.py.
 * tests/test_oracle.py pins both functions below to those fixtures.
 *
 *   oracle_attention_exact   follows lightglue_pytorch_no_plugin/lightglue.py:82-84
 *       query = query / 8; qk = softmax(query @ key^T, -1); out = qk @ value
 *     with fp64 accumulation (reference order: scale the query first, then the
 *     product, then a max-subtracted softmax, then the PV product).
 *
 *   oracle_attention_tiled   follows the kernel structure of the reference's
 *     FA2 kernel (lightglue_attention_plugin/attention_headdim_64_fp16in_fp32out.cu:398-703):
 *     64-key tiles, running row max m and running sum l, rescale by
 *     exp(m_prev - m_new) per tile, P rounded to fp16 before the PV product
 *     (…fp32out.cu:562-573), masked tail tile (…:473-492), final 1/l (…:667-673).
 *     fp32 arithmetic. Used to show that the tiled online formulation agrees with
 *     the exact one within the fp16-P rounding.
 *
 * Layout: Q [bh][nq][64], K/V [bh][nkv][64], O [bh][nq][64], float32, contiguous.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define HD 64

/* fp32 -> fp16 -> fp32, round-to-nearest-even (normal and subnormal range; no NaN inputs). */
static float round_f16(float x) {
    union { float f; uint32_t u; } in = {x};
    uint32_t sign = in.u & 0x80000000u;
    float a = fabsf(x);
    if (a >= 65520.0f) { union { uint32_t u; float f; } o = {sign | 0x7f800000u}; return o.f; }
    if (a < 6.103515625e-05f) {            /* fp16 subnormal: quantum 2^-24 */
        float q = nearbyintf(a * 16777216.0f) / 16777216.0f;
        return sign ? -q : q;
    }
    /* normal: keep 11 significant bits, RNE on the dropped 13 bits */
    union { float f; uint32_t u; } v = {a};
    uint32_t lsb = (v.u >> 13) & 1u;
    v.u += 0x0fffu + lsb;
    v.u &= ~0x1fffu;
    v.u |= sign;
    return v.f;
}

void oracle_round_f16(float* x, int64_t n) {
    for (int64_t i = 0; i < n; ++i) x[i] = round_f16(x[i]);
}

void oracle_attention_exact(const float* q, const float* k, const float* v, float* o,
                            int bh, int nq, int nkv) {
    double* s = (double*)malloc(sizeof(double) * (size_t)(nkv > 0 ? nkv : 1));
    for (int h = 0; h < bh; ++h) {
        const float* Q = q + (size_t)h * nq * HD;
        const float* K = k + (size_t)h * nkv * HD;
        const float* V = v + (size_t)h * nkv * HD;
        float* O = o + (size_t)h * nq * HD;
        for (int i = 0; i < nq; ++i) {
            double mx = -INFINITY;
            for (int j = 0; j < nkv; ++j) {
                double acc = 0.0;
                for (int d = 0; d < HD; ++d) acc += ((double)Q[i * HD + d] / 8.0) * (double)K[j * HD + d];
                s[j] = acc;
                if (acc > mx) mx = acc;
            }
            double sum = 0.0;
            for (int j = 0; j < nkv; ++j) { s[j] = exp(s[j] - mx); sum += s[j]; }
            for (int d = 0; d < HD; ++d) {
                double acc = 0.0;
                for (int j = 0; j < nkv; ++j) acc += s[j] * (double)V[j * HD + d];
                O[i * HD + d] = (float)(acc / sum);
            }
        }
    }
    free(s);
}

void oracle_attention_tiled(const float* q, const float* k, const float* v, float* o,
                            int bh, int nq, int nkv) {
    const int T = 64;
    float s[64], p[64], acc[HD];
    for (int h = 0; h < bh; ++h) {
        const float* Q = q + (size_t)h * nq * HD;
        const float* K = k + (size_t)h * nkv * HD;
        const float* V = v + (size_t)h * nkv * HD;
        float* O = o + (size_t)h * nq * HD;
        for (int i = 0; i < nq; ++i) {
            float m = -INFINITY, l = 0.0f;
            for (int d = 0; d < HD; ++d) acc[d] = 0.0f;
            for (int t0 = 0; t0 < nkv; t0 += T) {
                const int tn = (nkv - t0 < T) ? nkv - t0 : T;
                float tmax = -INFINITY;
                for (int j = 0; j < T; ++j) {
                    if (j >= tn) { s[j] = -INFINITY; continue; }   /* masked tail */
                    float a = 0.0f;
                    for (int d = 0; d < HD; ++d) a += Q[i * HD + d] * K[(t0 + j) * HD + d];
                    s[j] = a * 0.125f;
                    if (s[j] > tmax) tmax = s[j];
                }
                const float m_new = (tmax > m) ? tmax : m;
                const float alpha = expf(m - m_new);
                for (int d = 0; d < HD; ++d) acc[d] *= alpha;
                float ls = 0.0f;
                for (int j = 0; j < T; ++j) {
                    p[j] = expf(s[j] - m_new);
                    ls += p[j];
                    p[j] = round_f16(p[j]);
                }
                l = l * alpha + ls;
                m = m_new;
                for (int j = 0; j < tn; ++j)
                    for (int d = 0; d < HD; ++d) acc[d] += p[j] * V[(t0 + j) * HD + d];
            }
            const float inv = 1.0f / l;
            for (int d = 0; d < HD; ++d) O[i * HD + d] = acc[d] * inv;
        }
    }
}
