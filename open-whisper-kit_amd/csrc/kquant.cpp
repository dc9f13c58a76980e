// K-quant super-blocks (ref ggml/src/ggml-common.h:255-320, ggml/src/ggml-quants.c:703-1877):
// element decoding, the virtual-block expansion for k_gemm_q16 and the reference's row
// dequantization (token embedding rows). See kquant.h for the layout.
#include "kquant.h"

#include <cmath>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace owk {

namespace {

constexpr int QK = 256;

float h2f(const uint8_t * p) {
    uint16_t u;
    memcpy(&u, p, 2);
    return f16_to_f32_host(u);
}

// ref get_scale_min_k4 (ggml-quants.c:703-710): 6-bit scale and min j of q4_K / q5_K
void scale_min_k4(int j, const uint8_t * q, int & sc, int & m) {
    if (j < 4) {
        sc = q[j] & 63;
        m = q[j + 4] & 63;
    } else {
        sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
    }
}

// ref dequantize_row_q3_K (ggml-quants.c:1128-1151): the 12 scale bytes -> 16 6-bit values
void q3_scales(const uint8_t * s12, int8_t out[16]) {
    uint32_t aux[4];
    memcpy(aux, s12, 12);
    const uint32_t k1 = 0x03030303u, k2 = 0x0f0f0f0fu, tmp = aux[2];
    aux[2] = ((aux[0] >> 4) & k2) | (((tmp >> 4) & k1) << 4);
    aux[3] = ((aux[1] >> 4) & k2) | (((tmp >> 6) & k1) << 4);
    aux[0] = (aux[0] & k2) | (((tmp >> 0) & k1) << 4);
    aux[1] = (aux[1] & k2) | (((tmp >> 2) & k1) << 4);
    memcpy(out, aux, 16);
}

// one super-block: integer value q[p] of every element, the integer scale s16[j] and min m16[j]
// of every 16-wide group (32-wide formats: the group's sub-block), the f16 super-block scales
struct SB {
    int q[QK];
    int s16[16], m16[16];
    float d, dmin;
};

void decode(int fmt, const uint8_t * b, SB & o) {
    o.dmin = 0.0f;
    for (int j = 0; j < 16; ++j) o.m16[j] = 0;
    switch (fmt) {
        case QF_Q2_K: {  // scales[16], qs[64], d, dmin
            const uint8_t * sc = b, * qs = b + 16;
            o.d = h2f(b + 80);
            o.dmin = h2f(b + 82);
            for (int p = 0; p < QK; ++p) {
                const int c = p / 128, r = p % 128, j = r / 32, half = (r % 32) / 16, l = r % 16;
                o.q[p] = (qs[32 * c + l + 16 * half] >> (2 * j)) & 3;
            }
            for (int j = 0; j < 16; ++j) {
                o.s16[j] = sc[j] & 0xF;
                o.m16[j] = sc[j] >> 4;
            }
            break;
        }
        case QF_Q3_K: {  // hmask[32], qs[64], scales[12], d
            const uint8_t * hm = b, * qs = b + 32;
            int8_t s[16];
            q3_scales(b + 96, s);
            o.d = h2f(b + 108);
            for (int p = 0; p < QK; ++p) {
                const int c = p / 128, r = p % 128, j = r / 32, half = (r % 32) / 16, l = r % 16;
                const int lo = (qs[32 * c + l + 16 * half] >> (2 * j)) & 3;
                const int mbit = 1 << (4 * c + j);
                o.q[p] = lo - ((hm[l + 16 * half] & mbit) ? 0 : 4);
            }
            for (int j = 0; j < 16; ++j) o.s16[j] = s[j] - 32;
            break;
        }
        case QF_Q4_K:
        case QF_Q5_K: {  // d, dmin, scales[12], (q5_K: qh[32]), qs[128]
            o.d = h2f(b);
            o.dmin = h2f(b + 2);
            const uint8_t * sc = b + 4;
            const uint8_t * qh = fmt == QF_Q5_K ? b + 16 : nullptr;
            const uint8_t * qs = fmt == QF_Q5_K ? b + 48 : b + 16;
            for (int p = 0; p < QK; ++p) {
                const int c = p / 64, half = (p % 64) / 32, l = p % 32;
                const uint8_t byte = qs[32 * c + l];
                int q = half ? byte >> 4 : byte & 0xF;
                if (qh && (qh[l] & (1 << (2 * c + half)))) q += 16;
                o.q[p] = q;
            }
            for (int j = 0; j < 8; ++j) {
                int s, m;
                scale_min_k4(j, sc, s, m);
                o.s16[2 * j] = o.s16[2 * j + 1] = s;
                o.m16[2 * j] = o.m16[2 * j + 1] = m;
            }
            break;
        }
        case QF_Q6_K: {  // ql[128], qh[64], scales[16] int8, d
            const uint8_t * ql = b, * qh = b + 128;
            const int8_t * sc = (const int8_t *) (b + 192);
            o.d = h2f(b + 208);
            for (int p = 0; p < QK; ++p) {
                const int c = p / 128, k = (p % 128) / 32, l = p % 32;
                const uint8_t lb = ql[64 * c + l + ((k & 1) ? 32 : 0)];
                const int lo = k < 2 ? (lb & 0xF) : (lb >> 4);
                const int hi = (qh[32 * c + l] >> (2 * k)) & 3;
                o.q[p] = (lo | (hi << 4)) - 32;
            }
            for (int j = 0; j < 16; ++j) o.s16[j] = sc[j];
            break;
        }
        default: throw std::runtime_error("kquant: not a K-quant format");
    }
}

} // namespace

int kq_block_bytes(int fmt) {
    switch (fmt) {
        case QF_Q2_K: return 84;
        case QF_Q3_K: return 110;
        case QF_Q4_K: return 144;
        case QF_Q5_K: return 176;
        case QF_Q6_K: return 210;
    }
    throw std::runtime_error("kquant: bad format");
}

int kq_ggml_type(int fmt) {
    if (!qf_is_k(fmt)) throw std::runtime_error("kquant: bad format");
    return 10 + (fmt - QF_Q2_K);
}

int kq_layout(int fmt) {
    if (!qf_is_k(fmt)) throw std::runtime_error("kquant: bad format");
    return fmt == QF_Q3_K ? 1 : fmt == QF_Q6_K ? 2 : 0;
}

int kq_kx(int fmt, int K) {
    if (K % QK) throw std::runtime_error("kquant: row length not a multiple of 256");
    static const int per[3] = {288, 256, 512};
    return K / QK * per[kq_layout(fmt)];
}

void kq_expand_host(int fmt, const uint8_t * blocks, int N, int K, uint16_t * wi, float * dwt, int npad) {
    const int nsb = K / QK, kx = kq_kx(fmt, K), nkb = kx / 32, lay = kq_layout(fmt), bb = kq_block_bytes(fmt);
    if (npad < N) throw std::runtime_error("kquant: npad");
    for (int kb = 0; kb < nkb; ++kb)
        for (int n = N; n < npad; ++n) dwt[(size_t) kb * npad + n] = 0.0f;
    SB s;
    for (int n = 0; n < N; ++n) {
        uint16_t * w = wi + (size_t) n * kx;
        memset(w, 0, (size_t) kx * 2);
        for (int sb = 0; sb < nsb; ++sb) {
            decode(fmt, blocks + ((size_t) n * nsb + sb) * bb, s);
            if (lay == 0) {
                uint16_t * o = w + sb * 288;
                for (int p = 0; p < QK; ++p) o[p] = f32_to_f16_host((float) (s.s16[p / 16] * s.q[p]));
                for (int j = 0; j < 16; ++j) o[256 + j] = f32_to_f16_host((float) s.m16[j]);
                const int kb0 = sb * 9;
                for (int b = 0; b < 8; ++b) dwt[(size_t) (kb0 + b) * npad + n] = s.d;
                dwt[(size_t) (kb0 + 8) * npad + n] = -s.dmin;  // ref: dmin = -y.d * x.dmin
            } else if (lay == 1) {
                uint16_t * o = w + sb * 256;
                for (int p = 0; p < QK; ++p) o[p] = f32_to_f16_host((float) (s.s16[p / 16] * s.q[p]));
                for (int b = 0; b < 8; ++b) dwt[(size_t) (sb * 8 + b) * npad + n] = s.d;
            } else {
                uint16_t * o = w + sb * 512;
                for (int p = 0; p < QK; ++p) o[(p / 16) * 32 + p % 16] = f32_to_f16_host((float) s.q[p]);
                for (int j = 0; j < 16; ++j) dwt[(size_t) (sb * 16 + j) * npad + n] = s.d * (float) s.s16[j];
            }
        }
    }
}

void kq_dequant_row_host(int fmt, const uint8_t * blocks, int K, float * y) {
    const int nsb = K / QK, bb = kq_block_bytes(fmt);
    if (K % QK) throw std::runtime_error("kquant: row length not a multiple of 256");
    SB s;
    for (int sb = 0; sb < nsb; ++sb, y += QK) {
        decode(fmt, blocks + (size_t) sb * bb, s);
        for (int p = 0; p < QK; ++p) {
            const int j = p / 16;
            switch (fmt) {
                case QF_Q2_K:  // dl * q - ml (ref 784-812), contracted
                case QF_Q4_K:  // d1 * q - m1 (ref 1352-1373), contracted
                case QF_Q5_K: {
                    const float dl = s.d * (float) s.s16[j], ml = s.dmin * (float) s.m16[j];
                    y[p] = fmaf(dl, (float) s.q[p], -ml);
                    break;
                }
                case QF_Q3_K: y[p] = (s.d * (float) s.s16[j]) * (float) s.q[p]; break;  // dl * q (ref 1128-1170)
                case QF_Q6_K: y[p] = s.d * (float) s.s16[j] * (float) s.q[p]; break;    // d * sc * q (ref 1762-1789)
            }
        }
    }
}

} // namespace owk
