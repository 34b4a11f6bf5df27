/*
 * ngp_oracle.c — CPU restatement of the reference's hot-path kernels.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker for the HIP path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it. Nothing in torch-ngp_amd/ links or calls it; the product path has no CPU
 * fallback.
 *
 * Each function restates one reference CUDA kernel (file:line cited) as a
 * sequential loop. Floating-point order follows the reference expressions,
 * with fmaf()/fma() exactly where nvcc's default contraction fuses them and the
 * HIP kernels write them; built with -ffp-contract=off so nothing else fuses.
 * fp16 storage is emulated with explicit round-to-nearest-even conversions, so
 * `Half += float` rounds the product and then the sum (c10::Half semantics).
 * Integer outputs (sample counts, offsets, Morton codes, bitfields) and the
 * grid-encoder / marching float outputs are therefore reproducible bit for bit.
 *
 * The reference's only pinned artefacts for this path are the pure-torch
 * oracles in its testing/ directory (SHEncoder_torch, MLP) and trunc_exp; the
 * fixtures under tests/golden/ pin this file against them (see
 * tests/golden/make_golden.py). The CUDA kernels themselves cannot be built
 * here (no nvcc; CUTLASS submodule absent) — see DESIGN.md "Oracle".
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------- fp16 emulation (IEEE binary16, RNE) ---------------- */
uint16_t oracle_f2h(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t exp = (x >> 23) & 0xffu;
    uint32_t mant = x & 0x7fffffu;
    if (exp == 0xffu) return (uint16_t)(sign | 0x7c00u | (mant ? (0x200u | (mant >> 13)) : 0u));
    const int e = (int)exp - 127 + 15;
    if (e >= 0x1f) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        const int shift = 14 - e;
        uint32_t hm = mant >> shift;
        const uint32_t rem = mant & ((1u << shift) - 1u);
        const uint32_t halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (hm & 1u))) hm++;
        return (uint16_t)(sign | hm);
    }
    uint16_t h = (uint16_t)(sign | ((uint32_t)e << 10) | (mant >> 13));
    const uint32_t rem = mant & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return h;
}

float oracle_h2f(uint16_t h) {
    const uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1fu;
    uint32_t mant = h & 0x3ffu;
    uint32_t x;
    if (exp == 0) {
        if (mant == 0) {
            x = sign;
        } else {
            int e = -1;
            do { e++; mant <<= 1; } while (!(mant & 0x400u));
            x = sign | ((uint32_t)(127 - 15 - e) << 23) | ((mant & 0x3ffu) << 13);
        }
    } else if (exp == 0x1f) {
        x = sign | 0x7f800000u | (mant << 13);
    } else {
        x = sign | ((exp + 127 - 15) << 23) | (mant << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

void oracle_f2h_array(const float* in, uint16_t* out, size_t n) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_f2h(in[i]);
}
void oracle_h2f_array(const uint16_t* in, float* out, size_t n) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_h2f(in[i]);
}

/* ---------------- grid encoder (gridencoder/src/gridencoder.cu) ---------------- */

enum { DT_F32 = 0, DT_F16 = 1, DT_F64 = 2 };

/* scale = exp2f(level * S) * H - 1 (gridencoder.cu:138), exp2 evaluated in
 * double and rounded, identically to the HIP launcher. */
static float level_scale(uint32_t level, float S, uint32_t H) {
    const float ls = (float)level * S;
    const float e = (float)exp2((double)ls);
    return e * (float)H - 1.0f;
}

static uint32_t fast_hash(const uint32_t* pos, uint32_t D) {
    static const uint32_t primes[7] = {1u, 2654435761u, 805459861u, 3674653429u, 2097192037u,
                                       1434869437u, 2165219737u};
    uint32_t r = 0;
    for (uint32_t i = 0; i < D; ++i) r ^= pos[i] * primes[i];
    return r;
}

/* get_grid_index (gridencoder.cu:66-84), entry index (not times C) */
static uint32_t grid_index(uint32_t gridtype, int align_corners, uint32_t hs, uint32_t res,
                           const uint32_t* pos, uint32_t D) {
    uint32_t stride = 1, index = 0;
    for (uint32_t d = 0; d < D && stride <= hs; d++) {
        index += pos[d] * stride;
        stride *= align_corners ? res : (res + 1);
    }
    if (gridtype == 0 && stride > hs) index = fast_hash(pos, D);
    return index % hs;
}

static double load_v(const void* p, size_t i, int dt) {
    if (dt == DT_F32) return ((const float*)p)[i];
    if (dt == DT_F16) return oracle_h2f(((const uint16_t*)p)[i]);
    return ((const double*)p)[i];
}

static void store_v(void* p, size_t i, double v, int dt) {
    if (dt == DT_F32) ((float*)p)[i] = (float)v;
    else if (dt == DT_F16) ((uint16_t*)p)[i] = oracle_f2h((float)v);
    else ((double*)p)[i] = v;
}

/* scalar_t accumulate res += a * b with the reference's rounding */
static double mac_v(double res, double a, double b, int dt) {
    if (dt == DT_F32) return fmaf((float)a, (float)b, (float)res);
    if (dt == DT_F16) {
        const float prod = oracle_h2f(oracle_f2h((float)a * (float)b));
        return oracle_h2f(oracle_f2h((float)res + prod));
    }
    return fma(a, b, res);
}

static float smoothstep(float v) { return v * v * (3.0f - 2.0f * v); }
static float smoothstep_derivative(float v) { return 6 * v * (1.0f - v); }

/* kernel_grid (gridencoder.cu:87-242). out_layout 0: [L,B,C]; 1: [B,L*C].
 * Linear-mode dy_dx uses pos_deriv = 1 for every dimension (the reference
 * zero-initialises d >= 1, :143; documented divergence). */
int oracle_grid_encode_forward(const float* inputs, const void* emb, const int32_t* offsets,
                               void* outputs, uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                               float S, uint32_t H, void* dy_dx, uint32_t gridtype,
                               int align_corners, uint32_t interp, int dt, int out_layout) {
    if (D < 1 || D > 7 || C < 1 || C > 8) return -1;
    for (uint32_t level = 0; level < L; ++level) {
        const uint32_t off0 = (uint32_t)offsets[level];
        const uint32_t hs = (uint32_t)offsets[level + 1] - off0;
        const float scale = level_scale(level, S, H);
        const uint32_t res = (uint32_t)ceil(scale) + 1u;
        for (uint32_t b = 0; b < B; ++b) {
            const size_t obase = out_layout == 0 ? ((size_t)level * B + b) * C : ((size_t)b * L + level) * C;
            const float* x = inputs + (size_t)b * D;
            int oob = 0;
            for (uint32_t d = 0; d < D; ++d)
                if (x[d] < 0 || x[d] > 1) oob = 1;
            if (oob) {
                for (uint32_t c = 0; c < C; ++c) store_v(outputs, obase + c, 0.0, dt);
                if (dy_dx)
                    for (uint32_t i = 0; i < D * C; ++i) store_v(dy_dx, (size_t)b * D * L * C + level * D * C + i, 0.0, dt);
                continue;
            }
            float pos[8], pd[8];
            uint32_t pg[8];
            for (uint32_t d = 0; d < D; ++d) {
                pos[d] = fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
                pg[d] = (uint32_t)floorf(pos[d]);
                pos[d] -= (float)pg[d];
                pd[d] = 1.0f;
                if (interp == 1) {
                    pd[d] = smoothstep_derivative(pos[d]);
                    pos[d] = smoothstep(pos[d]);
                }
            }
            double resv[8] = {0};
            for (uint32_t idx = 0; idx < (1u << D); ++idx) {
                float w = 1;
                uint32_t pl[8];
                for (uint32_t d = 0; d < D; ++d) {
                    if ((idx & (1u << d)) == 0) { w *= 1 - pos[d]; pl[d] = pg[d]; }
                    else { w *= pos[d]; pl[d] = pg[d] + 1; }
                }
                const uint32_t e = grid_index(gridtype, align_corners, hs, res, pl, D);
                for (uint32_t c = 0; c < C; ++c)
                    resv[c] = mac_v(resv[c], w, load_v(emb, ((size_t)off0 + e) * C + c, dt), dt);
            }
            for (uint32_t c = 0; c < C; ++c) store_v(outputs, obase + c, resv[c], dt);
            if (dy_dx) {
                for (uint32_t gd = 0; gd < D; ++gd) {
                    double rg[8] = {0};
                    for (uint32_t idx = 0; idx < (1u << (D - 1)); ++idx) {
                        float w = scale;
                        uint32_t pl[8];
                        for (uint32_t nd = 0; nd < D - 1; ++nd) {
                            const uint32_t d = nd >= gd ? nd + 1 : nd;
                            if ((idx & (1u << nd)) == 0) { w *= 1 - pos[d]; pl[d] = pg[d]; }
                            else { w *= pos[d]; pl[d] = pg[d] + 1; }
                        }
                        pl[gd] = pg[gd];
                        const uint32_t il = grid_index(gridtype, align_corners, hs, res, pl, D);
                        pl[gd] = pg[gd] + 1;
                        const uint32_t ir = grid_index(gridtype, align_corners, hs, res, pl, D);
                        for (uint32_t c = 0; c < C; ++c) {
                            const double vr = load_v(emb, ((size_t)off0 + ir) * C + c, dt);
                            const double vl = load_v(emb, ((size_t)off0 + il) * C + c, dt);
                            double a;
                            if (dt == DT_F64) a = (double)w * (vr - vl);
                            else a = (double)(w * (float)(vr - vl));
                            rg[c] = mac_v(rg[c], a, (double)pd[gd], dt);
                        }
                    }
                    for (uint32_t c = 0; c < C; ++c)
                        store_v(dy_dx, (size_t)b * D * L * C + level * D * C + gd * C + c, rg[c], dt);
                }
            }
        }
    }
    return 0;
}

/* kernel_grid_backward (gridencoder.cu:245-337) as an exact float64 scatter.
 * Each contribution is the value the reference adds: for fp16 storage,
 * (half)(w * grad) (:325); for fp32, the fp32 product w * grad. grad_emb is a
 * float64 [sum_T, C] accumulator (the GPU's unordered atomics are compared to
 * it with a tolerance). */
int oracle_grid_encode_backward(const void* grad, const float* inputs, const int32_t* offsets,
                                double* grad_emb, uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                                float S, uint32_t H, uint32_t gridtype, int align_corners,
                                uint32_t interp, int dt, int grad_layout) {
    for (uint32_t level = 0; level < L; ++level) {
        const uint32_t off0 = (uint32_t)offsets[level];
        const uint32_t hs = (uint32_t)offsets[level + 1] - off0;
        const float scale = level_scale(level, S, H);
        const uint32_t res = (uint32_t)ceil(scale) + 1u;
        for (uint32_t b = 0; b < B; ++b) {
            const float* x = inputs + (size_t)b * D;
            int oob = 0;
            for (uint32_t d = 0; d < D; ++d)
                if (x[d] < 0 || x[d] > 1) oob = 1;
            if (oob) continue;
            float pos[8];
            uint32_t pg[8];
            for (uint32_t d = 0; d < D; ++d) {
                pos[d] = fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
                pg[d] = (uint32_t)floorf(pos[d]);
                pos[d] -= (float)pg[d];
                if (interp == 1) pos[d] = smoothstep(pos[d]);
            }
            const size_t gbase = grad_layout == 0 ? ((size_t)level * B + b) * C : ((size_t)b * L + level) * C;
            for (uint32_t idx = 0; idx < (1u << D); ++idx) {
                float w = 1;
                uint32_t pl[8];
                for (uint32_t d = 0; d < D; ++d) {
                    if ((idx & (1u << d)) == 0) { w *= 1 - pos[d]; pl[d] = pg[d]; }
                    else { w *= pos[d]; pl[d] = pg[d] + 1; }
                }
                const uint32_t e = grid_index(gridtype, align_corners, hs, res, pl, D);
                for (uint32_t c = 0; c < C; ++c) {
                    const double g = load_v(grad, gbase + c, dt);
                    double contrib;
                    if (dt == DT_F16) contrib = oracle_h2f(oracle_f2h(w * (float)g));
                    else if (dt == DT_F32) contrib = (double)(w * (float)g);
                    else contrib = (double)w * g;
                    grad_emb[((size_t)off0 + e) * C + c] += contrib;
                }
            }
        }
    }
    return 0;
}

/* kernel_grad_tv (gridencoder.cu:503-607): float or double table; every
 * point's per-entry contribution w * results * rsqrt(idelta + 1e-9) is formed
 * in the table's type (nvcc contracts idelta += v * v to an fma) and summed
 * into a float64 image (the reference's atomics are unordered). */
int oracle_grad_tv(const void* inputs, const void* grid, double* grad, const int32_t* offsets, float weight,
                   uint32_t B, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H, uint32_t gridtype,
                   int align_corners, int dt) {
    if (dt == DT_F16) return -1;
    for (uint32_t level = 0; level < L; ++level) {
        const uint32_t off0 = (uint32_t)offsets[level];
        const uint32_t hs = (uint32_t)offsets[level + 1] - off0;
        const float scale = level_scale(level, S, H);
        const uint32_t res = (uint32_t)ceil(scale) + 1u;
        for (uint32_t b = 0; b < B; ++b) {
            int oob = 0;
            for (uint32_t d = 0; d < D; ++d) {
                const double x = load_v(inputs, (size_t)b * D + d, dt);
                if (x < 0 || x > 1) oob = 1;
            }
            if (oob) continue;
            uint32_t pg[8];
            for (uint32_t d = 0; d < D; ++d) {
                const double x = load_v(inputs, (size_t)b * D + d, dt);
                /* inputs[d] * scale + 0.5 in scalar_t (fma under nvcc), then floorf */
                const float pos = dt == DT_F32 ? fmaf((float)x, scale, align_corners ? 0.0f : 0.5f)
                                               : (float)fma(x, (double)scale, align_corners ? 0.0 : 0.5);
                pg[d] = (uint32_t)floorf(pos);
            }
            const uint32_t index = grid_index(gridtype, align_corners, hs, res, pg, D);
            for (uint32_t c = 0; c < C; ++c) {
                double results = 0, idelta = 0;
                float rf = 0, idf = 0;
                const double g0 = load_v(grid, ((size_t)off0 + index) * C + c, dt);
                for (uint32_t d = 0; d < D; ++d) {
                    const uint32_t cur = pg[d];
                    for (int side = 0; side < 2; ++side) {
                        if (side == 0 ? !(cur < res) : !(cur > 0)) continue;
                        pg[d] = side == 0 ? cur + 1 : cur - 1;
                        const uint32_t nb = grid_index(gridtype, align_corners, hs, res, pg, D);
                        const double gv = g0 - load_v(grid, ((size_t)off0 + nb) * C + c, dt);
                        if (dt == DT_F32) {
                            const float gf = (float)g0 - (float)load_v(grid, ((size_t)off0 + nb) * C + c, dt);
                            rf += gf;
                            idf = fmaf(gf, gf, idf);
                        } else {
                            results += gv;
                            idelta = fma(gv, gv, idelta);
                        }
                        pg[d] = cur;
                    }
                }
                double contrib;
                if (dt == DT_F32) {
                    const float w = weight / (float)(2 * D);
                    contrib = (double)(w * rf * (1.0f / sqrtf(idf + 1e-9f)));
                } else {
                    const double w = (double)(weight / (float)(2 * D));
                    contrib = w * results * (double)(1.0f / sqrtf((float)(idelta + (double)1e-9f)));
                }
                grad[((size_t)off0 + index) * C + c] += contrib;
            }
        }
    }
    return 0;
}

/* kernel_input_backward (gridencoder.cu:340-366) */
int oracle_grid_input_backward(const void* grad, const void* dy_dx, void* grad_inputs, uint32_t B,
                               uint32_t D, uint32_t C, uint32_t L, int dt, int grad_layout) {
    for (uint32_t b = 0; b < B; ++b)
        for (uint32_t d = 0; d < D; ++d) {
            double r = 0.0;
            for (uint32_t l = 0; l < L; ++l)
                for (uint32_t c = 0; c < C; ++c) {
                    const size_t gi = grad_layout == 0 ? ((size_t)l * B + b) * C + c : ((size_t)b * L + l) * C + c;
                    r = mac_v(r, load_v(grad, gi, dt), load_v(dy_dx, (size_t)b * L * D * C + l * D * C + d * C + c, dt), dt);
                }
            store_v(grad_inputs, (size_t)b * D + d, r, dt);
        }
    return 0;
}

/* ---------------- ray marching (raymarching/src/raymarching.cu) ---------------- */

static float clampf_(float x, float lo, float hi) { return fminf(hi, fmaxf(lo, x)); }
static float signf_(float x) { return copysignf(1.0f, x); }

static int frexp_level(float mx, int maxl) {
    int e = 0;
    if (mx != 0.0f) frexpf(mx, &e);
    if (e < 0) e = 0;
    if (e > maxl) e = maxl;
    return e;
}

static uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
static uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2);
}
static uint32_t morton3_inv(uint32_t x) {
    x = x & 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

void oracle_morton3D(const int32_t* coords, uint32_t N, int32_t* idx) {
    for (uint32_t n = 0; n < N; ++n) idx[n] = (int32_t)morton3(coords[n * 3], coords[n * 3 + 1], coords[n * 3 + 2]);
}
void oracle_morton3D_invert(const int32_t* idx, uint32_t N, int32_t* coords) {
    for (uint32_t n = 0; n < N; ++n) {
        const uint32_t v = (uint32_t)idx[n];
        coords[n * 3] = (int32_t)morton3_inv(v);
        coords[n * 3 + 1] = (int32_t)morton3_inv(v >> 1);
        coords[n * 3 + 2] = (int32_t)morton3_inv(v >> 2);
    }
}
void oracle_packbits(const float* grid, uint32_t N, float thresh, uint8_t* bits) {
    for (uint32_t n = 0; n < N; ++n) {
        uint8_t v = 0;
        for (int i = 0; i < 8; ++i) v |= (grid[(size_t)n * 8 + i] > thresh) ? (uint8_t)(1u << i) : 0;
        bits[n] = v;
    }
}

/* kernel_near_far_from_aabb (raymarching.cu:91-145) */
void oracle_near_far_from_aabb(const float* ro, const float* rd, const float* aabb, uint32_t N,
                               float min_near, float* nears, float* fars) {
    for (uint32_t n = 0; n < N; ++n) {
        const float ox = ro[n * 3], oy = ro[n * 3 + 1], oz = ro[n * 3 + 2];
        const float rdx = 1 / rd[n * 3], rdy = 1 / rd[n * 3 + 1], rdz = 1 / rd[n * 3 + 2];
        float near = (aabb[0] - ox) * rdx, far = (aabb[3] - ox) * rdx;
        if (near > far) { float c = near; near = far; far = c; }
        float ny = (aabb[1] - oy) * rdy, fy = (aabb[4] - oy) * rdy;
        if (ny > fy) { float c = ny; ny = fy; fy = c; }
        if (near > fy || ny > far) { nears[n] = fars[n] = FLT_MAX; continue; }
        if (ny > near) near = ny;
        if (fy < far) far = fy;
        float nz = (aabb[2] - oz) * rdz, fz = (aabb[5] - oz) * rdz;
        if (nz > fz) { float c = nz; nz = fz; fz = c; }
        if (near > fz || nz > far) { nears[n] = fars[n] = FLT_MAX; continue; }
        if (nz > near) near = nz;
        if (fz < far) far = fz;
        if (near < min_near) near = min_near;
        nears[n] = near;
        fars[n] = far;
    }
}

typedef struct {
    float bound, dt_gamma, dt_min, dt_max, rH, H3;
    uint32_t max_steps, C, H;
} MarchK;

static MarchK march_k(float bound, float dt_gamma, uint32_t max_steps, uint32_t C, uint32_t H) {
    MarchK k;
    const float SQRT3 = 1.7320508075688772f;
    k.bound = bound;
    k.dt_gamma = dt_gamma;
    k.dt_min = 2 * SQRT3 / (float)max_steps;
    k.dt_max = 2 * SQRT3 * (float)(1u << (C - 1)) / (float)H;
    k.rH = 1 / (float)H;
    k.H3 = (float)(H * H * H);
    k.max_steps = max_steps;
    k.C = C;
    k.H = H;
    return k;
}

/* one step of the marching loop (raymarching.cu:359-400); returns occupancy,
 * advances t over an empty cell, and reports the sample */
static int march_step(const float* o, const float* d, const float* rd, const MarchK* k,
                      const uint8_t* grid, float* t, float* s) {
    const float x = clampf_(fmaf(*t, d[0], o[0]), -k->bound, k->bound);
    const float y = clampf_(fmaf(*t, d[1], o[1]), -k->bound, k->bound);
    const float z = clampf_(fmaf(*t, d[2], o[2]), -k->bound, k->bound);
    const float dt = clampf_(*t * k->dt_gamma, k->dt_min, k->dt_max);
    const int maxl = (int)k->C - 1;
    const float mxp = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    const float mxd = dt * (float)k->H * 0.5f;
    const int lp = frexp_level(mxp, maxl), ld = frexp_level(mxd, maxl);
    const int level = lp > ld ? lp : ld;
    const float mip_bound = fminf(ldexpf(1.0f, level), k->bound);
    const float mip_rbound = 1 / mip_bound;
    const float Hm1 = (float)(k->H - 1);
    const int nx = (int)clampf_(0.5f * fmaf(x, mip_rbound, 1.0f) * (float)k->H, 0.0f, Hm1);
    const int ny = (int)clampf_(0.5f * fmaf(y, mip_rbound, 1.0f) * (float)k->H, 0.0f, Hm1);
    const int nz = (int)clampf_(0.5f * fmaf(z, mip_rbound, 1.0f) * (float)k->H, 0.0f, Hm1);
    const uint32_t index = (uint32_t)((float)level * k->H3 + (float)morton3((uint32_t)nx, (uint32_t)ny, (uint32_t)nz));
    s[0] = x; s[1] = y; s[2] = z; s[3] = dt;
    if (grid[index / 8] & (1u << (index % 8))) return 1;
    const float tx = ((((float)nx + 0.5f + 0.5f * signf_(d[0])) * k->rH * 2 - 1) * mip_bound - x) * rd[0];
    const float ty = ((((float)ny + 0.5f + 0.5f * signf_(d[1])) * k->rH * 2 - 1) * mip_bound - y) * rd[1];
    const float tz = ((((float)nz + 0.5f + 0.5f * signf_(d[2])) * k->rH * 2 - 1) * mip_bound - z) * rd[2];
    const float tt = *t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    do {
        *t += clampf_(*t * k->dt_gamma, k->dt_min, k->dt_max);
    } while (*t < tt);
    return 0;
}

/* kernel_march_rays_train (raymarching.cu:311-480) with rays processed in
 * index order (ray_index = n; point offsets = prefix sum in ray order). */
int oracle_march_rays_train(const float* ro, const float* rdir, const uint8_t* grid, float bound,
                            float dt_gamma, uint32_t max_steps, uint32_t N, uint32_t C, uint32_t H,
                            uint32_t M, const float* nears, const float* fars, float* xyzs,
                            float* dirs, float* deltas, int32_t* rays, int32_t* counter,
                            const float* noises) {
    const MarchK k = march_k(bound, dt_gamma, max_steps, C, H);
    uint32_t point_base = (uint32_t)counter[0];
    for (uint32_t n = 0; n < N; ++n) {
        const float* o = ro + (size_t)n * 3;
        const float* d = rdir + (size_t)n * 3;
        const float rd[3] = {1 / d[0], 1 / d[1], 1 / d[2]};
        const float near = nears[n], far = fars[n];
        const float t0 = fmaf(clampf_(near * k.dt_gamma, k.dt_min, k.dt_max), noises[n], near);
        float t = t0, s[4];
        uint32_t num_steps = 0;
        while (t < far && num_steps < k.max_steps) {
            if (march_step(o, d, rd, &k, grid, &t, s)) {
                num_steps++;
                t += s[3];
            }
        }
        const uint32_t point_index = point_base;
        point_base += num_steps;
        rays[n * 3] = (int32_t)n;
        rays[n * 3 + 1] = (int32_t)point_index;
        rays[n * 3 + 2] = (int32_t)num_steps;
        if (num_steps == 0 || point_index + num_steps > M) continue;
        t = t0;
        float last_t = t;
        uint32_t step = 0;
        float* xyz = xyzs + (size_t)point_index * 3;
        float* dir = dirs + (size_t)point_index * 3;
        float* dl = deltas + (size_t)point_index * 2;
        while (t < far && step < num_steps) {
            if (march_step(o, d, rd, &k, grid, &t, s)) {
                xyz[0] = s[0]; xyz[1] = s[1]; xyz[2] = s[2];
                dir[0] = d[0]; dir[1] = d[1]; dir[2] = d[2];
                t += s[3];
                dl[0] = s[3];
                dl[1] = t - last_t;
                last_t = t;
                xyz += 3; dir += 3; dl += 2;
                step++;
            }
        }
    }
    counter[0] = (int32_t)point_base;
    counter[1] += (int32_t)N;
    return 0;
}

/* kernel_march_rays (raymarching.cu:709-814) */
int oracle_march_rays(uint32_t n_alive, uint32_t n_step, const int32_t* rays_alive,
                      const float* rays_t, const float* ro, const float* rdir, float bound,
                      float dt_gamma, uint32_t max_steps, uint32_t C, uint32_t H,
                      const uint8_t* grid, const float* nears, const float* fars, float* xyzs,
                      float* dirs, float* deltas, const float* noises) {
    const MarchK k = march_k(bound, dt_gamma, max_steps, C, H);
    (void)nears;
    for (uint32_t n = 0; n < n_alive; ++n) {
        const int index = rays_alive[n];
        const float* o = ro + (size_t)index * 3;
        const float* d = rdir + (size_t)index * 3;
        const float rd[3] = {1 / d[0], 1 / d[1], 1 / d[2]};
        float t = rays_t[index];
        const float far = fars[index];
        t = fmaf(clampf_(t * k.dt_gamma, k.dt_min, k.dt_max), noises[n], t);
        float last_t = t, s[4];
        uint32_t step = 0;
        float* xyz = xyzs + (size_t)n * n_step * 3;
        float* dir = dirs + (size_t)n * n_step * 3;
        float* dl = deltas + (size_t)n * n_step * 2;
        while (t < far && step < n_step) {
            if (march_step(o, d, rd, &k, grid, &t, s)) {
                xyz[0] = s[0]; xyz[1] = s[1]; xyz[2] = s[2];
                dir[0] = d[0]; dir[1] = d[1]; dir[2] = d[2];
                t += s[3];
                dl[0] = s[3];
                dl[1] = t - last_t;
                last_t = t;
                xyz += 3; dir += 3; dl += 2;
                step++;
            }
        }
    }
    return 0;
}

/* kernel_composite_rays_train_forward (raymarching.cu:500-577) */
int oracle_composite_rays_train_forward(const float* sigmas, const float* rgbs, const float* deltas,
                                        const int32_t* rays, uint32_t M, uint32_t N, float T_thresh,
                                        float* weights_sum, float* depth, float* image) {
    for (uint32_t n = 0; n < N; ++n) {
        const uint32_t index = (uint32_t)rays[n * 3], offset = (uint32_t)rays[n * 3 + 1];
        const uint32_t num_steps = (uint32_t)rays[n * 3 + 2];
        if (num_steps == 0 || offset + num_steps > M) {
            weights_sum[index] = 0; depth[index] = 0;
            image[index * 3] = image[index * 3 + 1] = image[index * 3 + 2] = 0;
            continue;
        }
        float T = 1.0f, r = 0, g = 0, b = 0, ws = 0, t = 0, dd = 0;
        for (uint32_t s = 0; s < num_steps; ++s) {
            const size_t i = (size_t)offset + s;
            const float alpha = 1.0f - expf(-sigmas[i] * deltas[i * 2]);
            const float weight = alpha * T;
            r = fmaf(weight, rgbs[i * 3], r);
            g = fmaf(weight, rgbs[i * 3 + 1], g);
            b = fmaf(weight, rgbs[i * 3 + 2], b);
            t += deltas[i * 2 + 1];
            dd = fmaf(weight, t, dd);
            ws += weight;
            T *= 1.0f - alpha;
            if (T < T_thresh) break;
        }
        weights_sum[index] = ws; depth[index] = dd;
        image[index * 3] = r; image[index * 3 + 1] = g; image[index * 3 + 2] = b;
    }
    return 0;
}

/* kernel_composite_rays_train_backward (raymarching.cu:601-691) */
int oracle_composite_rays_train_backward(const float* gws, const float* gdepth, const float* gimg,
                                         const float* sigmas, const float* rgbs, const float* deltas,
                                         const int32_t* rays, const float* ws_in, const float* depth,
                                         const float* image, uint32_t M, uint32_t N, float T_thresh,
                                         float* grad_sigmas, float* grad_rgbs) {
    for (uint32_t n = 0; n < N; ++n) {
        const uint32_t index = (uint32_t)rays[n * 3], offset = (uint32_t)rays[n * 3 + 1];
        const uint32_t num_steps = (uint32_t)rays[n * 3 + 2];
        if (num_steps == 0 || offset + num_steps > M) continue;
        const float gr = gimg[index * 3], gg = gimg[index * 3 + 1], gb = gimg[index * 3 + 2];
        const float gd = gdepth[index], gw = gws[index];
        const float rf = image[index * 3], gf = image[index * 3 + 1], bf = image[index * 3 + 2];
        const float wsf = ws_in[index], df = depth[index];
        float T = 1.0f, r = 0, g = 0, b = 0, t = 0, dd = 0;
        for (uint32_t s = 0; s < num_steps; ++s) {
            const size_t i = (size_t)offset + s;
            const float c0 = rgbs[i * 3], c1 = rgbs[i * 3 + 1], c2 = rgbs[i * 3 + 2];
            const float d0 = deltas[i * 2];
            const float alpha = 1.0f - expf(-sigmas[i] * d0);
            const float weight = alpha * T;
            r = fmaf(weight, c0, r);
            g = fmaf(weight, c1, g);
            b = fmaf(weight, c2, b);
            t += deltas[i * 2 + 1];
            dd = fmaf(weight, t, dd);
            T *= 1.0f - alpha;
            grad_rgbs[i * 3] = gr * weight;
            grad_rgbs[i * 3 + 1] = gg * weight;
            grad_rgbs[i * 3 + 2] = gb * weight;
            grad_sigmas[i] = d0 * (gr * (T * c0 - (rf - r)) + gg * (T * c1 - (gf - g)) +
                                   gb * (T * c2 - (bf - b)) + gd * (T * t - (df - dd)) +
                                   gw * (1 - wsf));
            if (T < T_thresh) break;
        }
    }
    return 0;
}

/* kernel_composite_rays (raymarching.cu:827-914), in place */
int oracle_composite_rays(uint32_t n_alive, uint32_t n_step, float T_thresh, int32_t* rays_alive,
                          float* rays_t, const float* sigmas, const float* rgbs, const float* deltas,
                          float* weights_sum, float* depth, float* image) {
    for (uint32_t n = 0; n < n_alive; ++n) {
        const int index = rays_alive[n];
        const float* sg = sigmas + (size_t)n * n_step;
        const float* cl = rgbs + (size_t)n * n_step * 3;
        const float* dl = deltas + (size_t)n * n_step * 2;
        float t = rays_t[index], wsum = weights_sum[index], d = depth[index];
        float r = image[index * 3], g = image[index * 3 + 1], b = image[index * 3 + 2];
        uint32_t step = 0;
        while (step < n_step) {
            const float d0 = dl[step * 2];
            if (d0 == 0) break;
            const float alpha = 1.0f - expf(-sg[step] * d0);
            const float T = 1 - wsum;
            const float weight = alpha * T;
            wsum += weight;
            t += dl[step * 2 + 1];
            d = fmaf(weight, t, d);
            r = fmaf(weight, cl[step * 3], r);
            g = fmaf(weight, cl[step * 3 + 1], g);
            b = fmaf(weight, cl[step * 3 + 2], b);
            if (T < T_thresh) break;
            step++;
        }
        if (step < n_step) rays_alive[n] = -1;
        else rays_t[index] = t;
        weights_sum[index] = wsum; depth[index] = d;
        image[index * 3] = r; image[index * 3 + 1] = g; image[index * 3 + 2] = b;
    }
    return 0;
}
