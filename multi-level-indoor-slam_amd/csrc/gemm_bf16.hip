// bf16 "NT" GEMM for the ViT-B/14 projections with fused epilogues (gfx950).
//
//   C[m, n] = epilogue( sum_k A[m, k] * W[n, k] )
//
// A: activations, bf16 row-major [M, K]; W: nn.Linear weight, bf16 row-major [N, K].
// Both operands are K-contiguous, which is exactly what the 16x16x32 bf16 MFMA
// fragments want (8 consecutive k per lane).  The product is computed transposed
// (D = W . A^T per 16x16 tile) so that each lane ends up owning 4 consecutive output
// columns of one token row: epilogue stores are 8-byte bf16 / 16-byte f32 vectors.
//
// Tile 128 x 128 x 64, 256 threads (2 x 2 waves of 64 x 64), register-staged double
// buffer in LDS (64 KiB -> 2 workgroups per CU), st_16x32-style XOR swizzle
// (chunk ^ (row >> 1) & 7) that makes every ds_read_b128 fragment read conflict-free,
// XCD-aware bijective block remap so the N-tiles of one M-panel share an L2.
//
// Requirements (checked by the host launcher): K % 64 == 0, N % 128 == 0,
// 16-byte aligned A / W rows.  M is arbitrary (rows >= M are clamped on load and
// masked on store).
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;  // one operand tile, 16 KiB

__device__ __forceinline__ int swz_off(int row, int chunk) {
    return row * (BK * 2) + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// ------------------------------------------------------------------ epilogues
struct EpiF32 {  // plain f32 store (testing)
    float* C; int ldc;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        *reinterpret_cast<float4*>(C + (size_t)m * ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
    }
};

struct EpiBiasF32 {  // y = acc + b  -> f32
    float* C; int ldc; const float* bias;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        *reinterpret_cast<float4*>(C + (size_t)m * ldc + n) = make_float4(v[0] + b.x, v[1] + b.y, v[2] + b.z, v[3] + b.w);
    }
};

// y = acc + b as a bf16 pair hi = bf16(y), lo = bf16(y - hi) (y = hi + lo to 2^-17),
// k-step-major [N / 16][rows][16] so a 32-row MFMA fragment load is one contiguous
// 1 KiB (LightGlue's assignment similarity, lightglue.hip k_asg_sim)
struct EpiBiasSplitBF16 {
    bf16_t* H; bf16_t* L; int rows; const float* bias;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        const float y0 = v[0] + b.x, y1 = v[1] + b.y, y2 = v[2] + b.z, y3 = v[3] + b.w;
        const uint32_t h01 = pack_bf16x2(y0, y1), h23 = pack_bf16x2(y2, y3);
        const float r0 = y0 - __uint_as_float(h01 << 16), r1 = y1 - __uint_as_float(h01 & 0xffff0000u);
        const float r2 = y2 - __uint_as_float(h23 << 16), r3 = y3 - __uint_as_float(h23 & 0xffff0000u);
        const size_t o = ((size_t)(n >> 4) * rows + m) * 16 + (n & 15);
        *reinterpret_cast<uint2*>(H + o) = make_uint2(h01, h23);
        *reinterpret_cast<uint2*>(L + o) = make_uint2(pack_bf16x2(r0, r1), pack_bf16x2(r2, r3));
    }
};

// LoFTR's coarse similarity from the split-bf16 product: S[m][n] = (acc / 256) / 0.1 as
// the exact-f32 path scales it (mlg_similarity_f32_loftr), columns n < ncols; rows of lds
// floats (lds % 4 == 0, >= ncols: the GEMM's N is padded to the 256-column tile), the
// columns [ncols, lds) written -inf so that 16-B row reads see no similarity there (a
// frame of L % 4 != 0 cells, e.g. 720 x 536: L = 6030, lds = 6032)
struct EpiSimLoFTR {
    float* S; int lds; int ncols;
    struct Col {};
    struct Row {};
    struct Pre {};
    __device__ Col col(int) const { return {}; }
    __device__ Row row(int) const { return {}; }
    __device__ Pre pre(int, int, const Col&, const Row&) const { return {}; }
    __device__ static float sc(float a) { return (a * (1.0f / 256.0f)) / 0.1f; }
    __device__ void store(int m, int n, float a, float b, float c, float d) const {
        float* row = S + (size_t)m * lds;
        if (n + 3 < ncols) {
            *reinterpret_cast<float4*>(row + n) = make_float4(a, b, c, d);
        } else if (n < lds) {  // n % 4 == 0 and lds % 4 == 0: the quad lies inside the row
            *reinterpret_cast<float4*>(row + n) =
                make_float4(n < ncols ? a : -INFINITY, n + 1 < ncols ? b : -INFINITY, n + 2 < ncols ? c : -INFINITY,
                            n + 3 < ncols ? d : -INFINITY);
        }
    }
    // staged form (k_gemm256s): the scaled products staged as f32 rows, written as whole
    // 256-B row pieces (no read of S: load4 is a no-op)
    static constexpr int STAGED = 2;
    __device__ float4 stage4(const f32x4& v, const Col&) const {
        return make_float4(sc(v[0]), sc(v[1]), sc(v[2]), sc(v[3]));
    }
    __device__ float4 load4(int, int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
    __device__ void put4(int m, int n, float4, const float4& y) const { store(m, n, y.x, y.y, y.z, y.w); }
    __device__ void apply(int m, int n, const f32x4& v, const Col&, const Row&, const Pre&) const {
        store(m, n, sc(v[0]), sc(v[1]), sc(v[2]), sc(v[3]));
    }
    __device__ void operator()(int m, int n, const f32x4& v) const { apply(m, n, v, Col{}, Row{}, Pre{}); }
};

struct EpiBiasBF16 {  // y = acc + b  -> bf16
    bf16_t* C; int ldc; const float* bias;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        uint2 o;
        o.x = pack_bf16x2(v[0] + b.x, v[1] + b.y);
        o.y = pack_bf16x2(v[2] + b.z, v[3] + b.w);
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) = o;
    }
};

// y = gelu(acc + b) -> bf16   (mlp.fc1 + nn.GELU(); the erf form as common.h gelu_poly2,
// no transcendental: the A & S 7.1.26 form's v_rcp + v_exp per element made this epilogue
// the VALU bound of fc1)
struct EpiBiasGeluBF16 {
    bf16_t* C; int ldc; const float* bias;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        const f32x2 g01 = gelu_poly2(f32x2{v[0] + b.x, v[1] + b.y});
        const f32x2 g23 = gelu_poly2(f32x2{v[2] + b.z, v[3] + b.w});
        uint2 o;
        o.x = pack_bf16x2(g01.x, g01.y);
        o.y = pack_bf16x2(g23.x, g23.y);
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) = o;
    }
};

// y = gelu(acc + b) as the split pair: hi = bf16(y) at column n, lo = bf16(y - hi) at
// column n + lo_col of the same row (the [hi | lo] A rows of the split fc2 GEMM).  GELU as
// common.h gelu_poly2 (|error| <= 1e-6, below the pair's 2^-17 relative representation
// error for |y| > 0.13; erff here made fc1 epilogue-bound: MLG_SPLIT_GELU_ERF=1 keeps it
// for A/B)
#ifndef MLG_SPLIT_GELU_ERF
#define MLG_SPLIT_GELU_ERF 0
#endif
#ifndef MLG_EPI_PROBE
#define MLG_EPI_PROBE 0  // timing-probe builds only (results wrong): 4 no fc1 stores, 8 no GELU
#endif
struct EpiBiasGeluSplit {
    bf16_t* C; int ldc; int lo_col; const float* bias;
    __device__ static float gelu(float x) { return 0.5f * x * (1.0f + erff(x * 0.7071067811865476f)); }
    // batched form (epi_tile): column data, row data, per-fragment prefetch, apply
    struct Col { float4 b; };
    struct Row { size_t key = 0; };  // (staged form: unused)
    struct Pre {};
    __device__ Col col(int n) const { return {*reinterpret_cast<const float4*>(bias + n)}; }
    __device__ Row row(int) const { return {}; }
    __device__ Pre pre(int, int, const Col&, const Row&) const { return {}; }
    // staged form (k_gemm256s): the pair computed in the fragment layout, written from an
    // LDS image as whole rows (put)
    static constexpr int STAGED = 1;
    __device__ bool staged_wave(int) const { return true; }
    __device__ void stage2(const f32x4& v, const Col& c, uint2& h, uint2& l) const {
        const float4 b = c.b;
#if MLG_SPLIT_GELU_ERF
        split_bf16x4(gelu(v[0] + b.x), gelu(v[1] + b.y), gelu(v[2] + b.z), gelu(v[3] + b.w), h, l);
#else
        const f32x2 g01 = gelu_poly2(f32x2{v[0] + b.x, v[1] + b.y});
        const f32x2 g23 = gelu_poly2(f32x2{v[2] + b.z, v[3] + b.w});
        split_bf16x4(g01.x, g01.y, g23.x, g23.y, h, l);
#endif
    }
    __device__ void put(int m, int n, int plane, size_t, const uint4& d) const {
        *reinterpret_cast<uint4*>(C + (size_t)m * ldc + (plane ? lo_col : 0) + n) = d;
    }
    __device__ void apply(int m, int n, const f32x4& v, const Col& c, const Row&, const Pre&) const {
        const float4 b = c.b;
        uint2 h, l;
#if MLG_SPLIT_GELU_ERF
        split_bf16x4(gelu(v[0] + b.x), gelu(v[1] + b.y), gelu(v[2] + b.z), gelu(v[3] + b.w), h, l);
#elif MLG_EPI_PROBE & 8  // timing probe only: no GELU
        split_bf16x4(v[0] + b.x, v[1] + b.y, v[2] + b.z, v[3] + b.w, h, l);
#else
        const f32x2 g01 = gelu_poly2(f32x2{v[0] + b.x, v[1] + b.y});
        const f32x2 g23 = gelu_poly2(f32x2{v[2] + b.z, v[3] + b.w});
        split_bf16x4(g01.x, g01.y, g23.x, g23.y, h, l);
#endif
#if MLG_EPI_PROBE & 4  // timing probe only: stores kept alive by an impossible test
        if (h.x != 0x7f817f81u) return;
#endif
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) = h;
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + lo_col + n) = l;
    }
    __device__ void operator()(int m, int n, const f32x4& v) const { apply(m, n, v, col(n), Row{}, Pre{}); }
};

struct EpiResidual {  // X += gamma * (acc + b)   (attn.proj / mlp.fc2 + LayerScale + residual)
    float* X; int ldx; const float* bias; const float* gamma;
    struct Col { float4 b, g; };
    struct Row {};
    struct Pre { float4 x; };
    __device__ Col col(int n) const {
        return {*reinterpret_cast<const float4*>(bias + n), *reinterpret_cast<const float4*>(gamma + n)};
    }
    __device__ Row row(int) const { return {}; }
    __device__ Pre pre(int m, int n, const Col&, const Row&) const {
        return {*reinterpret_cast<const float4*>(X + (size_t)m * ldx + n)};
    }
    // staged form (k_gemm256s): acc + b staged as f32 rows, then x += gamma * (that) per row
    static constexpr int STAGED = 2;
    __device__ float4 stage4(const f32x4& v, const Col& c) const {
        return make_float4(v[0] + c.b.x, v[1] + c.b.y, v[2] + c.b.z, v[3] + c.b.w);
    }
    __device__ float4 load4(int m, int n) const { return *reinterpret_cast<const float4*>(X + (size_t)m * ldx + n); }
    __device__ void put4(int m, int n, float4 x, const float4& y) const {
        const float4 g = *reinterpret_cast<const float4*>(gamma + n);
        x.x += g.x * y.x;
        x.y += g.y * y.y;
        x.z += g.z * y.z;
        x.w += g.w * y.w;
        *reinterpret_cast<float4*>(X + (size_t)m * ldx + n) = x;
    }
    __device__ void apply(int m, int n, const f32x4& v, const Col& c, const Row&, const Pre& p) const {
        float4 x = p.x;
        x.x += c.g.x * (v[0] + c.b.x);
        x.y += c.g.y * (v[1] + c.b.y);
        x.z += c.g.z * (v[2] + c.b.z);
        x.w += c.g.w * (v[3] + c.b.w);
        *reinterpret_cast<float4*>(X + (size_t)m * ldx + n) = x;
    }
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const Col c = col(n);
        apply(m, n, v, c, Row{}, pre(m, n, c, Row{}));
    }
};

// qkv -> Q, K bf16 [12][B * Tpad][64] and V^T bf16 tiled [12][B * Tpad / 64][64 d][64 keys]
// (the layouts k_attention_varlen reads; image b is the segment b * Tpad of each head)
struct EpiQKV {
    bf16_t* Q; bf16_t* K; bf16_t* Vt; const float* bias; int T, Tpad, Np;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        const int bi = m / T, t = m - bi * T;
        const int which = n / 768, c = n - which * 768, h = c >> 6, d = c & 63;
        const size_t key = (size_t)bi * Tpad + t;
        if (which < 2) {
            uint2 o;
            o.x = pack_bf16x2(v[0] + b.x, v[1] + b.y);
            o.y = pack_bf16x2(v[2] + b.z, v[3] + b.w);
            *reinterpret_cast<uint2*>((which == 0 ? Q : K) + ((size_t)h * Np + key) * 64 + d) = o;
        } else {  // transposed per 64-key block so attention streams V^T rows (key-contiguous)
            bf16_t* p = Vt + (((size_t)h * (Np >> 6) + (key >> 6)) * 64 + d) * 64 + (key & 63);
            p[0] = f32_to_bf16(v[0] + b.x);
            p[64] = f32_to_bf16(v[1] + b.y);
            p[128] = f32_to_bf16(v[2] + b.z);
            p[192] = f32_to_bf16(v[3] + b.w);
        }
    }
};

// relu(acc + b) -> bf16, columns >= nvalid dropped (N padded to the tile width)
// EpiQKV for the split forward: hi planes as EpiQKV, lo planes lo_off elements further
struct EpiQKVSplit {
    bf16_t* Q; bf16_t* K; bf16_t* Vt; const float* bias; int T, Tpad, Np; size_t lo_off;
    struct Col { float4 b; };
    struct Row { size_t key; };
    struct Pre {};
    __device__ Col col(int n) const { return {*reinterpret_cast<const float4*>(bias + n)}; }
    __device__ Row row(int m) const {
        const int bi = m / T, t = m - bi * T;
        return {(size_t)bi * Tpad + t};
    }
    __device__ Pre pre(int, int, const Col&, const Row&) const { return {}; }
    __device__ void operator()(int m, int n, const f32x4& v) const { apply(m, n, v, col(n), row(m), Pre{}); }
    // staged form (k_gemm256s) for the Q / K waves (a wave's 64 columns are one head of one
    // of q, k, v): whole 128-B token rows of the head-major planes; V^T keeps apply
    static constexpr int STAGED = 1;
    __device__ bool staged_wave(int n) const { return n < 2 * 768; }
    __device__ void stage2(const f32x4& v, const Col& c, uint2& h, uint2& l) const {
        split_bf16x4(v[0] + c.b.x, v[1] + c.b.y, v[2] + c.b.z, v[3] + c.b.w, h, l);
    }
    __device__ void put(int, int n, int plane, size_t key, const uint4& dd) const {
        const int which = n / 768, c = n - which * 768, h = c >> 6, d = c & 63;
        *reinterpret_cast<uint4*>((which == 0 ? Q : K) + ((size_t)h * Np + key) * 64 + d + (plane ? lo_off : 0)) = dd;
    }
    __device__ void apply(int, int n, const f32x4& v, const Col& cd, const Row& rw, const Pre&) const {
        const float4 b = cd.b;
        const int which = n / 768, c = n - which * 768, h = c >> 6, d = c & 63;
        const size_t key = rw.key;
        uint2 hi, lo;
        split_bf16x4(v[0] + b.x, v[1] + b.y, v[2] + b.z, v[3] + b.w, hi, lo);
        if (which < 2) {
            bf16_t* p = (which == 0 ? Q : K) + ((size_t)h * Np + key) * 64 + d;
            *reinterpret_cast<uint2*>(p) = hi;
            *reinterpret_cast<uint2*>(p + lo_off) = lo;
        } else {
            bf16_t* p = Vt + (((size_t)h * (Np >> 6) + (key >> 6)) * 64 + d) * 64 + (key & 63);
            const uint32_t e[4] = {hi.x & 0xffffu, hi.x >> 16, hi.y & 0xffffu, hi.y >> 16};
            const uint32_t f[4] = {lo.x & 0xffffu, lo.x >> 16, lo.y & 0xffffu, lo.y >> 16};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                p[64 * i] = (bf16_t)e[i];
                p[64 * i + lo_off] = (bf16_t)f[i];
            }
        }
    }
};

struct EpiBiasReluBF16 {
    bf16_t* C; int ldc; const float* bias; int nvalid;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        if (n >= nvalid) return;
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        uint2 o;
        o.x = pack_bf16x2(fmaxf(v[0] + b.x, 0.f), fmaxf(v[1] + b.y, 0.f));
        o.y = pack_bf16x2(fmaxf(v[2] + b.z, 0.f), fmaxf(v[3] + b.w, 0.f));
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) = o;
    }
};

// X = relu((acc + b) + R) in f32 (R may alias X) and its bf16 copy (ResNet conv3 + shortcut)
struct EpiBiasAddRelu {
    const float* R; float* X; int ldx; bf16_t* C; const float* bias;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const float4 b = *reinterpret_cast<const float4*>(bias + n);
        const float4 r = *reinterpret_cast<const float4*>(R + (size_t)m * ldx + n);
        float4 x;
        x.x = fmaxf((v[0] + b.x) + r.x, 0.f);
        x.y = fmaxf((v[1] + b.y) + r.y, 0.f);
        x.z = fmaxf((v[2] + b.z) + r.z, 0.f);
        x.w = fmaxf((v[3] + b.w) + r.w, 0.f);
        *reinterpret_cast<float4*>(X + (size_t)m * ldx + n) = x;
        uint2 o;
        o.x = pack_bf16x2(x.x, x.y);
        o.y = pack_bf16x2(x.z, x.w);
        *reinterpret_cast<uint2*>(C + (size_t)m * ldx + n) = o;
    }
};

// Generic conv / linear epilogue (LoFTR, loftr.hip): y = acc (+ bias) (+ R[m, n]), then
// act 1 = ReLU, 2 = LeakyReLU(0.01), 3 = elu + 1 on columns < act_cols; stored as f32
// (X, ldx) and / or bf16 (C, ldc), either may be null.
#ifndef MLG_GEMM_ROW_STAGED
#define MLG_GEMM_ROW_STAGED 1  // 0: EpiConv fragment-at-a-time in k_gemm256 (A/B arm)
#endif
struct EpiConv {
    // row-major outputs / residual: k_gemm256 runs it from an LDS row image (whole-row
    // accesses) -- see row_staged below
    static constexpr bool ROW_STAGED = MLG_GEMM_ROW_STAGED;
    const float* bias; const float* R; int ldr; float* X; int ldx; bf16_t* C; int ldc; int act; int act_cols;
    float vdiv = 0.f;  // != 0: columns >= act_cols divided by it (LoFTR's values / v_length)
    __device__ void operator()(int m, int n, const f32x4& v) const {
        float y[4] = {v[0], v[1], v[2], v[3]};
        if (bias) {
            const float4 b = *reinterpret_cast<const float4*>(bias + n);
            y[0] += b.x; y[1] += b.y; y[2] += b.z; y[3] += b.w;
        }
        if (R) {
            const float4 r = *reinterpret_cast<const float4*>(R + (size_t)m * ldr + n);
            y[0] += r.x; y[1] += r.y; y[2] += r.z; y[3] += r.w;
        }
        if (act && n < act_cols) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (act == 1) y[i] = fmaxf(y[i], 0.f);
                else if (act == 2) y[i] = y[i] > 0.f ? y[i] : 0.01f * y[i];
                else y[i] = (y[i] > 0.f ? y[i] : expf(y[i]) - 1.f) + 1.f;  // elu(y) + 1, as torch
            }
        }
        if (vdiv != 0.f && n >= act_cols) {
#pragma unroll
            for (int i = 0; i < 4; ++i) y[i] = y[i] / vdiv;
        }
        if (X) *reinterpret_cast<float4*>(X + (size_t)m * ldx + n) = make_float4(y[0], y[1], y[2], y[3]);
        if (C) *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) =
            make_uint2(pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]));
    }
};

// LoFTR's FPN merge in the lateral 1x1 conv's epilogue: C = bf16((acc + bias) +
// up(src)), up = bilinear x2 (align_corners=True) of the coarser NHWC f32 map src [B, h,
// w, N] at output pixel m = (b, oy, ox) of the [B, 2h, 2w] grid -- the same expressions in
// the same order as k_lf_up_add reading the conv's f32 output, so the same bits, without
// the f32 lateral map's write and re-read.  Row-staged (whole-row stores).
struct EpiConvUp {
    static constexpr bool ROW_STAGED = true;
    const float* bias; const float* src; int h, w; bf16_t* C; int ldc;
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const int Ho = 2 * h, Wo = 2 * w;
        const int x = m % Wo, r = m / Wo, y = r % Ho, b = r / Ho;
        float l0 = v[0], l1 = v[1], l2 = v[2], l3 = v[3];  // no bias: as EpiConv, no add at all
        if (bias) {
            const float4 bb = *reinterpret_cast<const float4*>(bias + n);
            l0 += bb.x;
            l1 += bb.y;
            l2 += bb.z;
            l3 += bb.w;
        }
        const float sh = Ho > 1 ? (float)(h - 1) / (float)(Ho - 1) : 0.f;
        const float sw = Wo > 1 ? (float)(w - 1) / (float)(Wo - 1) : 0.f;
        const float fy = sh * (float)y, fx = sw * (float)x;
        const int y0 = (int)fy, x0 = (int)fx;
        const int y1 = y0 < h - 1 ? y0 + 1 : y0, x1 = x0 < w - 1 ? x0 + 1 : x0;
        const float ly1 = fy - (float)y0, lx1 = fx - (float)x0, ly0 = 1.f - ly1, lx0 = 1.f - lx1;
        const float* s0 = src + ((size_t)b * h * w) * ldc + n;
        const float4 v00 = *reinterpret_cast<const float4*>(s0 + ((size_t)y0 * w + x0) * ldc);
        const float4 v01 = *reinterpret_cast<const float4*>(s0 + ((size_t)y0 * w + x1) * ldc);
        const float4 v10 = *reinterpret_cast<const float4*>(s0 + ((size_t)y1 * w + x0) * ldc);
        const float4 v11 = *reinterpret_cast<const float4*>(s0 + ((size_t)y1 * w + x1) * ldc);
        const float o0 = lf_up_add1(l0, v00.x, v01.x, v10.x, v11.x, lx0, lx1, ly0, ly1);
        const float o1 = lf_up_add1(l1, v00.y, v01.y, v10.y, v11.y, lx0, lx1, ly0, ly1);
        const float o2 = lf_up_add1(l2, v00.z, v01.z, v10.z, v11.z, lx0, lx1, ly0, ly1);
        const float o3 = lf_up_add1(l3, v00.w, v01.w, v10.w, v11.w, lx0, lx1, ly0, ly1);
        *reinterpret_cast<uint2*>(C + (size_t)m * ldc + n) = make_uint2(pack_bf16x2(o0, o1), pack_bf16x2(o2, o3));
    }
};

struct EpiPatch {  // patch tokens: X[b, 1 + p, :] = acc + b + pos[1 + p]
    float* X; const float* bias; const float* pos; int P;  // P = patches per image
    struct Col { float4 b; };
    struct Row { int bi, p; };
    struct Pre { float4 q; };
    __device__ Col col(int n) const { return {*reinterpret_cast<const float4*>(bias + n)}; }
    __device__ Row row(int m) const {
        const int bi = m / P;
        return {bi, m - bi * P};
    }
    __device__ Pre pre(int, int n, const Col&, const Row& r) const {
        return {*reinterpret_cast<const float4*>(pos + (size_t)(1 + r.p) * 768 + n)};
    }
    __device__ void apply(int, int n, const f32x4& v, const Col& c, const Row& r, const Pre& pq) const {
        const float4 b = c.b, q = pq.q;
        *reinterpret_cast<float4*>(X + ((size_t)r.bi * (P + 1) + 1 + r.p) * 768 + n) =
            make_float4(v[0] + b.x + q.x, v[1] + b.y + q.y, v[2] + b.z + q.z, v[3] + b.w + q.w);
    }
    __device__ void operator()(int m, int n, const f32x4& v) const {
        const Col c = col(n);
        const Row r = row(m);
        apply(m, n, v, c, r, pre(m, n, c, r));
    }
};

// ---------------------------------------------------------------------- kernel
template <class Epi>
__global__ __launch_bounds__(256, 2) void k_gemm_nt(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K, int lda, int ldw, Epi epi) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nN = N / BN, nM = (M + BM - 1) / BM, nwg = nN * nM;
    // XCD-aware bijective remap: hardware blocks b, b+8, ... (one XCD) get consecutive
    // logical ids, so the N-tiles of an M-panel run on one XCD and share its L2.
    const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    const int mt = wgid / nN, nt = wgid - mt * nN;
    const int m0 = mt * BM, n0 = nt * BN;

    // staging: 1024 16-B chunks per operand tile, 4 per thread (rows tid>>3 + 32 i)
    const int srow = tid >> 3, sch = tid & 7;
    const bf16_t* pa = A + (size_t)min(m0 + srow, M - 1) * lda + sch * 8;
    const bf16_t* pw = W + (size_t)(n0 + srow) * ldw + sch * 8;
    const size_t a32 = (size_t)lda * 32, w32 = (size_t)ldw * 32;
    // rows >= M are clamped to M - 1 (their products are never stored)
    const int ar1 = min(m0 + srow + 32, M - 1) - min(m0 + srow, M - 1);
    const int ar2 = min(m0 + srow + 64, M - 1) - min(m0 + srow, M - 1);
    const int ar3 = min(m0 + srow + 96, M - 1) - min(m0 + srow, M - 1);
    const int so0 = swz_off(srow, sch), so1 = swz_off(srow + 32, sch);
    const int so2 = swz_off(srow + 64, sch), so3 = swz_off(srow + 96, sch);
    uint4 ra0, ra1, ra2, ra3, rw0, rw1, rw2, rw3;
#define GEMM_GLOAD(k0)                                                              \
    {                                                                               \
        ra0 = *reinterpret_cast<const uint4*>(pa + (k0));                           \
        ra1 = *reinterpret_cast<const uint4*>(pa + (size_t)ar1 * lda + (k0));       \
        ra2 = *reinterpret_cast<const uint4*>(pa + (size_t)ar2 * lda + (k0));       \
        ra3 = *reinterpret_cast<const uint4*>(pa + (size_t)ar3 * lda + (k0));       \
        rw0 = *reinterpret_cast<const uint4*>(pw + (k0));                           \
        rw1 = *reinterpret_cast<const uint4*>(pw + w32 + (k0));                     \
        rw2 = *reinterpret_cast<const uint4*>(pw + 2 * w32 + (k0));                 \
        rw3 = *reinterpret_cast<const uint4*>(pw + 3 * w32 + (k0));                 \
    }
#define GEMM_LSTORE(buf)                                                            \
    {                                                                               \
        char* b_ = smem + (buf) * 2 * TILE_BYTES;                                   \
        *reinterpret_cast<uint4*>(b_ + so0) = ra0;                                  \
        *reinterpret_cast<uint4*>(b_ + so1) = ra1;                                  \
        *reinterpret_cast<uint4*>(b_ + so2) = ra2;                                  \
        *reinterpret_cast<uint4*>(b_ + so3) = ra3;                                  \
        *reinterpret_cast<uint4*>(b_ + TILE_BYTES + so0) = rw0;                     \
        *reinterpret_cast<uint4*>(b_ + TILE_BYTES + so1) = rw1;                     \
        *reinterpret_cast<uint4*>(b_ + TILE_BYTES + so2) = rw2;                     \
        *reinterpret_cast<uint4*>(b_ + TILE_BYTES + so3) = rw3;                     \
    }
    (void)a32;

    const int wn = wave >> 1, wm = wave & 1;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / BK;
    GEMM_GLOAD(0);
    GEMM_LSTORE(0);
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) { GEMM_GLOAD((kt + 1) * BK); }
        const char* base = smem + cur * 2 * TILE_BYTES;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 af[4], wf[4];
            const int ch = s * 4 + (lane >> 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = wm * 64 + j * 16 + (lane & 15);
                af[j] = *reinterpret_cast<const bf16x8*>(base + swz_off(row, ch));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = wn * 64 + i * 16 + (lane & 15);
                wf[i] = *reinterpret_cast<const bf16x8*>(base + TILE_BYTES + swz_off(row, ch));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) { GEMM_LSTORE(cur ^ 1); }
        __syncthreads();
        cur ^= 1;
    }

#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4;
            const int m = m0 + wm * 64 + j * 16 + (lane & 15);
            if (m < M) epi(m, n, acc[i][j]);
        }
#undef GEMM_GLOAD
#undef GEMM_LSTORE
}

// ------------------------------------------------------- LDS-DMA kernels
// 128 x 256 x BK tile, 512 threads = 8 waves (2 along M x 4 along N, 64 x 64 each),
// STAGES LDS stages filled by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave-instruction), K-tile t+2 prefetched while t is computed.  The XOR swizzle
// (chunk ^ (row >> 1) & (chunks/row - 1), conflict-free for every ds_read_b128
// fragment read at BK = 32 and 64 -- checked by script) moves to the per-lane SOURCE
// address since the DMA writes lane-linear; fragment reads apply the same involution.
// Waits are counted (s_waitcnt vmcnt(#DMA per tile): the newest tile's DMAs stay in
// flight across the raw s_barrier); each stage is its own __shared__ object and the
// loop is unrolled by 3 so stage addresses are constants.
//   BK = 64: 3 x 48 KiB stages, one workgroup per CU.
//   BK = 32: 3 x 24 KiB stages, two workgroups per CU (16 waves): one workgroup's
//            epilogue / prologue overlaps the other's MFMA main loop.
namespace dma {
constexpr int BM = 128, BN = 256;
typedef __attribute__((address_space(3))) char lds_char;

// LDS byte address of a __shared__ object (the value M0 carries for LDS-DMA).
__device__ __forceinline__ unsigned lds_addr(char* p) { return (unsigned)(uintptr_t)(lds_char*)p; }

// One global_load_lds_dwordx4: 16 B per lane from `g` into LDS [m0 + 16 * lane].
// Issued through inline asm so hipcc's waitcnt pass does not conservatively drain
// vmcnt(0) before every fragment read of the other stages; all waits on these DMAs
// are the explicit counted s_waitcnt vmcnt of the pipeline.
// `s_nop 0`: the SALU-write-M0 -> LDS-DMA-read-M0 wait state, which hipcc pads for the
// builtin but not for an asm statement (it puts its s_mov_b32 m0 directly in front).
__device__ __forceinline__ void dma16(const void* g, unsigned m0) {
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}
// Same with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset.
__device__ __forceinline__ void dma16s(unsigned voff, const void* sbase, unsigned m0) {
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
}

template <int BK>
__device__ __forceinline__ int soff(int row, int chunk) {
    return row * (BK * 2) + ((chunk ^ ((row >> 1) & (BK / 8 - 1))) << 4);
}

template <class Epi, int BK>
__global__ __launch_bounds__(512, BK == 32 ? 4 : 2) void k_gemm(const bf16_t* __restrict__ A,
                                                                 const bf16_t* __restrict__ W, int M, int N, int K,
                                                                 int lda, int ldw, Epi epi) {
    constexpr int CH = BK / 8;                         // 16-B chunks per row
    constexpr int RPI = 64 / CH;                       // rows per DMA wave-instruction
    constexpr int NA = BM / RPI / 8, NB = BN / RPI / 8;  // DMAs per wave per K-tile
    constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
    constexpr int WAIT_NEWEST = 0xF70 | (NA + NB);     // s_waitcnt vmcnt(NA + NB)
    __shared__ __attribute__((aligned(16))) char st0[STAGE];
    __shared__ __attribute__((aligned(16))) char st1[STAGE];
    __shared__ __attribute__((aligned(16))) char st2[STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nN = N / BN, nM = (M + BM - 1) / BM, nwg = nN * nM;
    const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    const int mt = wgid / nN, nt = wgid - mt * nN;
    const int m0 = mt * BM, n0 = nt * BN;

    // DMA sources: wave w fills A row-groups NA*w .. and B row-groups NB*w .. (RPI rows each)
    const int lr = lane / CH, lp = lane % CH;
    const bf16_t* pa[NA];
    const bf16_t* pb[NB];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int row = (NA * wave + i) * RPI + lr;
        pa[i] = A + (size_t)min(m0 + row, M - 1) * lda + ((lp ^ ((row >> 1) & (CH - 1))) * 8);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int row = (NB * wave + i) * RPI + lr;
        pb[i] = W + (size_t)(n0 + row) * ldw + ((lp ^ ((row >> 1) & (CH - 1))) * 8);
    }
    const int da = NA * wave * 1024, db = A_BYTES + NB * wave * 1024;

#define DMA_ISSUE(ST, k0)                                                                                  \
    {                                                                                                      \
        const unsigned b_ = lds_addr(ST);                                                                  \
        _Pragma("unroll") for (int i = 0; i < NA; ++i) dma16(pa[i] + (k0), b_ + da + i * 1024);            \
        _Pragma("unroll") for (int i = 0; i < NB; ++i) dma16(pb[i] + (k0), b_ + db + i * 1024);            \
    }

    const int wm = wave & 1, wn = wave >> 1;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#define DMA_COMPUTE(ST)                                                                                    \
    _Pragma("unroll") for (int s = 0; s < BK / 32; ++s) {                                                  \
        bf16x8 af[4], wf[4];                                                                               \
        const int ch = s * 4 + (lane >> 4);                                                                \
        _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                                    \
            const int row = wm * 64 + j * 16 + (lane & 15);                                                \
            af[j] = *reinterpret_cast<const bf16x8*>((ST) + soff<BK>(row, ch));                            \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                    \
            const int row = wn * 64 + i * 16 + (lane & 15);                                                \
            wf[i] = *reinterpret_cast<const bf16x8*>((ST) + A_BYTES + soff<BK>(row, ch));                  \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 4; ++j)        \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);         \
    }

    // Every step issues its DMA unconditionally (past the last K-tile it re-reads the
    // last tile into a stage that is never read again): one code path, one wait count.
#define DMA_STEP(TT, CUR, NXT)                                                                             \
    {                                                                                                      \
        DMA_ISSUE(NXT, min((TT) + 2, nk - 1) * BK);                                                        \
        DMA_COMPUTE(CUR);                                                                                  \
        __builtin_amdgcn_s_waitcnt(WAIT_NEWEST);                                                           \
        __builtin_amdgcn_s_barrier();                                                                      \
    }

    const int nk = K / BK;  // multiple of 3 (checked by the launcher)
    DMA_ISSUE(st0, 0);
    DMA_ISSUE(st1, BK);
    __builtin_amdgcn_s_waitcnt(WAIT_NEWEST);
    __builtin_amdgcn_s_barrier();
    for (int t = 0; t < nk; t += 3) {
        DMA_STEP(t, st0, st2)
        DMA_STEP(t + 1, st1, st0)
        DMA_STEP(t + 2, st2, st1)
    }
    __builtin_amdgcn_s_waitcnt(0xF70);  // no DMA may still be writing LDS when the block retires
#undef DMA_STEP
#undef DMA_COMPUTE
#undef DMA_ISSUE

#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4;
            const int m = m0 + wm * 64 + j * 16 + (lane & 15);
            if (m < M) epi(m, n, acc[i][j]);
        }
}
// 256 x 256 x 64 tile, 8 waves (2 along M x 4 along N, 128 x 64 each: 32 accumulators),
// two 64 KiB LDS stages (K-tile t+1 lands while t is computed), one workgroup per CU,
// PERSISTENT: the grid is one workgroup per CU and each walks a contiguous range of
// output tiles of its XCD (N fastest, so the 32 workgroups of an XCD share A panels
// in that XCD's L2).  The last K-step of a tile already DMAs K-tile 0 of the next tile,
// so the next tile's first wait overlaps this tile's epilogue, and the epilogue's
// stores drain while the next tile's MFMAs run.  Twice the MFMAs per barrier and
// 0.375 fragment reads per MFMA (vs 0.5 at 64 x 64 per wave).
// Row-staged epilogue of a wave's RM x 64 block of a persistent 256-row tile (k_gemm256,
// k_conv256): the accumulators (16 x 16 fragments, lane = 4 consecutive columns of one
// row) go through IMG bytes of the dead LDS stage as f32 rows, PR rows a pass, 16-B chunks
// swizzled by the row; each lane then applies the epilogue to a float4 of one row, 16
// lanes per row, so the residual reads and the f32 / bf16 stores are whole 256-B / 128-B
// row pieces instead of 16 rows x 32-64 B per wave-instruction.  Same per-element math
// (the same epi() call): the same bits.  The caller syncs the workgroup before the stage
// is refilled.
template <class E, class = void>
struct row_staged { static constexpr bool value = false; };
template <class E>
struct row_staged<E, std::void_t<decltype(E::ROW_STAGED)>> { static constexpr bool value = E::ROW_STAGED; };

template <int RM, int IMG, class Epi, int JM>
__device__ __forceinline__ void gemm256_rows_epilogue(const Epi& epi, const f32x4 (&acc)[4][JM], char* img, int mw,
                                                      int nw, int M, int lane) {
    constexpr int PR = IMG >= 8192 ? 32 : 16, NP = RM / PR, JP = PR / 16;
    static_assert(RM == JM * 16 && RM % PR == 0 && PR * 256 <= IMG, "row-staged epilogue shape");
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int jj = 0; jj < JP; ++jj) {
            const int r = jj * 16 + (lane & 15);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ch = 4 * i + (lane >> 4);
                *reinterpret_cast<f32x4*>(img + r * 256 + ((ch ^ (r & 15)) << 4)) = acc[i][p * JP + jj];
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's image written
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < PR / 4; ++it) {
            const int L = it * 64 + lane, r = L >> 4, ch = L & 15;
            const int m = mw + p * PR + r;
            const f32x4 v = *reinterpret_cast<const f32x4*>(img + r * 256 + ((ch ^ (r & 15)) << 4));
            if (m < M) epi(m, nw + ch * 4, v);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // image read before the next pass writes it
        __builtin_amdgcn_wave_barrier();
    }
}

template <class Epi>
__global__ __launch_bounds__(512, 2) void k_gemm256(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                   int M, int N, int K, int lda, int ldw, Epi epi) {
    constexpr int BK = 64, TM = 256, TN = 256;
    constexpr int A_BYTES = TM * BK * 2, STAGE = (TM + TN) * BK * 2;  // 64 KiB
    constexpr int NA = 4, NB = 4;                                      // DMAs per wave per K-tile
    __shared__ __attribute__((aligned(16))) char st0[STAGE];
    __shared__ __attribute__((aligned(16))) char st1[STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nN = N / TN, nM = (M + TM - 1) / TM, ntiles = nN * nM;
    const int xcd = blockIdx.x & 7, per_xcd = gridDim.x >> 3;  // grid is a multiple of 8
    const int tx = (ntiles + 7) >> 3;
    const int tile_end = min((xcd + 1) * tx, ntiles);
    int tile = xcd * tx + (blockIdx.x >> 3);
    if (tile >= tile_end) return;

    const int lr = lane >> 3, lp = lane & 7;
    const int wm = wave & 1, wn = wave >> 1;
    const int da = NA * wave * 1024, db = A_BYTES + NB * wave * 1024;
    const int nk = K / BK;  // even (checked by the launcher)

    // DMA addressing: wave-uniform tile bases (SGPRs) + 32-bit per-lane byte offsets.
    // B offsets are the same for every tile (N % 256 == 0); A offsets change only for
    // the ragged last M-tile, whose rows are clamped to M - 1.
    unsigned ob[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int row = (NB * wave + i) * 8 + lr;
        ob[i] = (unsigned)(row * ldw + ((lp ^ ((row >> 1) & 7)) * 8)) * 2u;
    }
    auto a_offsets = [&](int t, unsigned* oa) {
        const int m0 = (t / nN) * TM;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int row = (NA * wave + i) * 8 + lr;
            oa[i] = (unsigned)((min(m0 + row, M - 1) - m0) * lda + ((lp ^ ((row >> 1) & 7)) * 8)) * 2u;
        }
    };
    auto a_base = [&](int t) { return A + (size_t)((t / nN) * TM) * lda; };
    auto b_base = [&](int t) { return W + (size_t)((t % nN) * TN) * ldw; };
    unsigned oa[NA];
    const bf16_t* sa = a_base(tile);
    const bf16_t* sb = b_base(tile);
    a_offsets(tile, oa);
#define D256_DMA(ST, OA, SA, SB, t)                                                                        \
    {                                                                                                      \
        const unsigned b_ = lds_addr(ST);                                                                  \
        const bf16_t* sa_ = (SA) + (t) * BK;                                                               \
        const bf16_t* sb_ = (SB) + (t) * BK;                                                               \
        _Pragma("unroll") for (int i = 0; i < NA; ++i) dma16s((OA)[i], sa_, b_ + da + i * 1024);           \
        _Pragma("unroll") for (int i = 0; i < NB; ++i) dma16s(ob[i], sb_, b_ + db + i * 1024);             \
    }
#define D256_COMPUTE(ST)                                                                                   \
    _Pragma("unroll") for (int s = 0; s < 2; ++s) {                                                        \
        bf16x8 af[8], wf[4];                                                                               \
        const int ch = s * 4 + (lane >> 4);                                                                \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                    \
            const int row = wn * 64 + i * 16 + (lane & 15);                                                \
            wf[i] = *reinterpret_cast<const bf16x8*>((ST) + A_BYTES + soff<64>(row, ch));                  \
        }                                                                                                  \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                    \
            const int row = wm * 128 + j * 16 + (lane & 15);                                               \
            af[j] = *reinterpret_cast<const bf16x8*>((ST) + soff<64>(row, ch));                            \
        }                                                                                                  \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) _Pragma("unroll") for (int i = 0; i < 4; ++i)        \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);         \
    }

    D256_DMA(st0, oa, sa, sb, 0);
    __builtin_amdgcn_s_waitcnt(0xF70);
    __builtin_amdgcn_s_barrier();
    for (; tile < tile_end; tile += per_xcd) {
        const int next = tile + per_xcd < tile_end ? tile + per_xcd : tile;
        unsigned na[NA];
        a_offsets(next, na);
        const bf16_t* nsa = a_base(next);
        const bf16_t* nsb = b_base(next);
        const int kn = next != tile ? 0 : nk - 1;  // K-tile of the last DMA (no next tile: harmless re-read)
        f32x4 acc[4][8];  // [n-tile][m-tile]
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < nk; t += 2) {
            D256_DMA(st1, oa, sa, sb, t + 1);
            D256_COMPUTE(st0);
            __builtin_amdgcn_s_waitcnt(0xF70);
            __builtin_amdgcn_s_barrier();
            if (t + 2 < nk) {
                D256_DMA(st0, oa, sa, sb, t + 2);
            } else {
                D256_DMA(st0, na, nsa, nsb, kn);  // K-tile 0 of the next output tile
            }
            D256_COMPUTE(st1);
            __builtin_amdgcn_s_waitcnt(0xF70);
            __builtin_amdgcn_s_barrier();
        }
        const int mt = tile / nN, m0 = mt * TM, n0 = (tile - mt * nN) * TN;
        if constexpr (row_staged<Epi>::value) {
            gemm256_rows_epilogue<TM / 2, STAGE / 8>(epi, acc, st1 + wave * (STAGE / 8), m0 + wm * 128, n0 + wn * 64,
                                                     M, lane);
            __syncthreads();  // every wave's image read: the next tile DMAs into st1
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4;
                    const int m = m0 + wm * 128 + j * 16 + (lane & 15);
                    if (m < M) epi(m, n, acc[i][j]);
                }
        }
#pragma unroll
        for (int i = 0; i < NA; ++i) oa[i] = na[i];
        sa = nsa;
        sb = nsb;
    }
    __builtin_amdgcn_s_waitcnt(0xF70);
#undef D256_COMPUTE
#undef D256_DMA
}

// Split-bf16 GEMM (MLG_VIT_SPLIT): C = epi(A_hi W_hi^T + A_hi W_lo^T + A_lo W_hi^T), f32
// accumulation.  A rows are [A_hi | A_lo] (K0 each, lda >= 2 K0), W rows [W_hi | W_lo]
// (ldw >= 2 K0).  The persistent, XCD-local 256 x 256 tile of k_gemm256 with K-steps of
// 32: one LDS stage holds the four 256 x 32 planes of a K-step (64 KiB, two stages), each
// wave reads its W_hi / W_lo / A_hi fragments, issues the hi*hi and lo*hi MFMAs, then
// reloads its A fragments as A_lo for the hi*lo MFMAs -- 96 MFMAs per 24 fragment reads
// per wave and K-step, and every operand byte fetched once (a K-concatenated [hi|lo|hi]
// GEMM re-reads A_hi and W_hi: 3 planes each instead of 2).
// Epi::STAGED (k_gemm256s): 1 = a bf16 hi / lo pair per element written from an LDS image
// as whole rows (stage2 / put), 2 = an f32 row update (stage4 / load4 / put4), 0 = none
template <class E, class = void>
struct staged_of { static constexpr int value = 0; };
template <class E>
struct staged_of<E, std::void_t<decltype(E::STAGED)>> { static constexpr int value = E::STAGED; };

// MLG_S256_PRIO: s_setprio(1) / (0) around each MFMA cluster of k_gemm256s (the guide's
// T5: hipcc then keeps the cluster between its barriers)
#ifndef MLG_S256_PRIO
#define MLG_S256_PRIO 1
#endif
#if MLG_S256_PRIO
#define S256_PRIO(p) __builtin_amdgcn_s_setprio(p)
#else
#define S256_PRIO(p) ((void)0)
#endif
template <class Epi>
__global__ __launch_bounds__(512, 1) void k_gemm256s(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K0, int lda, int ldw, Epi epi, int nb,
                                                    long sA, long sW) {
    constexpr int BK = 32, TM = 256, TN = 256;
    constexpr int PLANE = TM * BK * 2;  // 16 KiB: one 256 x 32 bf16 operand plane
    constexpr int STAGE = 4 * PLANE;    // A_hi, A_lo, W_hi, W_lo
    __shared__ __attribute__((aligned(16))) char st0[STAGE];
    __shared__ __attribute__((aligned(16))) char st1[STAGE];
    constexpr int STG = staged_of<Epi>::value;
    __shared__ size_t skey[STG == 1 ? 8 : 1][32];  // staged form: the pass's row keys per wave
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // nb > 1 (staged-f32 epilogues only): nb independent products of one shape in one
    // persistent launch, problem z at A + z sA, W + z sW, its output rows z M + m (the
    // LoFTR similarity of a pair group: one tile queue instead of a 2-3-tile tail per pair)
    const int nN = N / TN, nM = (M + TM - 1) / TM, nMN = nN * nM, ntiles = nb * nMN;
    const int xcd = blockIdx.x & 7, per_xcd = gridDim.x >> 3;
    const int tx = (ntiles + 7) >> 3;
    const int tile_end = min((xcd + 1) * tx, ntiles);
    int tile = xcd * tx + (blockIdx.x >> 3);
    if (tile >= tile_end) return;

    const int lr = lane >> 2, lp = lane & 3;  // 16 rows x 4 chunks of 16 B per DMA wave-instruction
    const int wm = wave & 1, wn = wave >> 1;
    const int nk = K0 / BK;  // even (checked by the launcher)
    const int drow = 2 * wave * 1024;  // this wave's 32 rows of every plane
    unsigned ob[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = (2 * wave + i) * 16 + lr;
        ob[i] = (unsigned)(row * ldw + ((lp ^ ((row >> 1) & 3)) * 8)) * 2u;
    }
    auto a_offsets = [&](int t, unsigned* oa) {
        const int m0 = ((t % nMN) / nN) * TM;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = (2 * wave + i) * 16 + lr;
            oa[i] = (unsigned)((min(m0 + row, M - 1) - m0) * lda + ((lp ^ ((row >> 1) & 3)) * 8)) * 2u;
        }
    };
    auto a_base = [&](int t) { return A + (t / nMN) * sA + (size_t)(((t % nMN) / nN) * TM) * lda; };
    auto b_base = [&](int t) { return W + (t / nMN) * sW + (size_t)((t % nN) * TN) * ldw; };
    unsigned oa[2];
    const bf16_t* sa = a_base(tile);
    const bf16_t* sb = b_base(tile);
    a_offsets(tile, oa);
#define S256_DMA(ST, OA, SA, SB, t)                                                                        \
    {                                                                                                      \
        const unsigned b_ = lds_addr(ST) + drow;                                                           \
        const bf16_t* ah_ = (SA) + (t) * BK;                                                               \
        const bf16_t* wh_ = (SB) + (t) * BK;                                                               \
        _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                                    \
            dma16s((OA)[i], ah_, b_ + i * 1024);                                                           \
            dma16s((OA)[i], ah_ + K0, b_ + PLANE + i * 1024);                                              \
            dma16s(ob[i], wh_, b_ + 2 * PLANE + i * 1024);                                                 \
            dma16s(ob[i], wh_ + K0, b_ + 3 * PLANE + i * 1024);                                            \
        }                                                                                                  \
    }
#define S256_COMPUTE(ST)                                                                                   \
    {                                                                                                      \
        bf16x8 af[8], wh[4], wl[4];                                                                        \
        const int ch = lane >> 4;                                                                          \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                    \
            const int row = wn * 64 + i * 16 + (lane & 15);                                                \
            wh[i] = *reinterpret_cast<const bf16x8*>((ST) + 2 * PLANE + soff<32>(row, ch));                \
            wl[i] = *reinterpret_cast<const bf16x8*>((ST) + 3 * PLANE + soff<32>(row, ch));                \
        }                                                                                                  \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                    \
            const int row = wm * 128 + j * 16 + (lane & 15);                                               \
            af[j] = *reinterpret_cast<const bf16x8*>((ST) + soff<32>(row, ch));                            \
        }                                                                                                  \
        S256_PRIO(1);                                                                                      \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) _Pragma("unroll") for (int i = 0; i < 4; ++i) {      \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[i], af[j], acc[i][j], 0, 0, 0);         \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[i], af[j], acc[i][j], 0, 0, 0);         \
        }                                                                                                  \
        S256_PRIO(0);                                                                                      \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                    \
            const int row = wm * 128 + j * 16 + (lane & 15);                                               \
            af[j] = *reinterpret_cast<const bf16x8*>((ST) + PLANE + soff<32>(row, ch));                    \
        }                                                                                                  \
        S256_PRIO(1);                                                                                      \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) _Pragma("unroll") for (int i = 0; i < 4; ++i)        \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[i], af[j], acc[i][j], 0, 0, 0);         \
        S256_PRIO(0);                                                                                      \
    }

    S256_DMA(st0, oa, sa, sb, 0);
    __builtin_amdgcn_s_waitcnt(0xF70);
    __builtin_amdgcn_s_barrier();
    for (; tile < tile_end; tile += per_xcd) {
        const int next = tile + per_xcd < tile_end ? tile + per_xcd : tile;
        unsigned na[2];
        a_offsets(next, na);
        const bf16_t* nsa = a_base(next);
        const bf16_t* nsb = b_base(next);
        const int kn = next != tile ? 0 : nk - 1;  // no next tile: harmless re-read
        f32x4 acc[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < nk; t += 2) {
            S256_DMA(st1, oa, sa, sb, t + 1);
            S256_COMPUTE(st0);
            __builtin_amdgcn_s_waitcnt(0xF70);
            __builtin_amdgcn_s_barrier();
            if (t + 2 < nk) {
                S256_DMA(st0, oa, sa, sb, t + 2);
            } else {
                S256_DMA(st0, na, nsa, nsb, kn);  // K-step 0 of the next output tile
            }
            S256_COMPUTE(st1);
            __builtin_amdgcn_s_waitcnt(0xF70);
            __builtin_amdgcn_s_barrier();
        }
        const int tz = tile / nMN, lt = tile - tz * nMN, mz = tz * M;
        const int mt = lt / nN, m0 = mt * TM, n0 = (lt - mt * nN) * TN;
        // batched epilogue: every column's (bias, ...) and every row's index data first, then
        // per column group the 8 fragments' global reads (the residual) before any of their
        // stores -- a fragment-at-a-time epilogue waited one L2 / HBM round trip per
        // fragment (its loads could not pass the previous fragment's stores), 32 per tile
        // A tile wholly inside M takes a branch-free form: a per-fragment `m < M` test made
        // every fragment its own basic block (no interleaving of their GELU chains, and a
        // conservative vmcnt wait at every block entry that serialised the stores).
        auto epilogue = [&](auto check) {
            constexpr bool CHECK = decltype(check)::value;
            typename Epi::Col cols[4];
            typename Epi::Row rows[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) cols[i] = epi.col(n0 + wn * 64 + i * 16 + (lane >> 4) * 4);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int m = m0 + wm * 128 + j * 16 + (lane & 15);
                rows[j] = epi.row(CHECK ? min(m, M - 1) : m);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4;
                typename Epi::Pre pre[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int m = m0 + wm * 128 + j * 16 + (lane & 15);
                    pre[j] = epi.pre(CHECK ? min(m, M - 1) : m, n, cols[i], rows[j]);
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int m = m0 + wm * 128 + j * 16 + (lane & 15);
                    if (!CHECK || m < M) epi.apply(m, n, acc[i][j], cols[i], rows[j], pre[j]);
                }
            }
        };
        // Staged form: the wave's 128 x 64 outputs in 4 passes of 32 rows through its 8 KiB
        // of the dead stage st1 (free until the next tile's second K-step DMA, after the
        // barrier below), then written as whole 128-B (bf16) / 256-B (f32) row pieces: the
        // fragment layout stores 16 rows x 32 B per wave-instruction, and those partial-line
        // stores cost a third of the fc1 GEMM (profiles/r04af_split_gemm_epilogue_probe.txt).
        if constexpr (STG == 1) {
            const int nw = n0 + wn * 64;
            if (epi.staged_wave(nw)) {
                char* img = st1 + wave * 8192;
                typename Epi::Col cols[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) cols[i] = epi.col(nw + i * 16 + (lane >> 4) * 4);
#pragma unroll
                for (int p = 0; p < 4; ++p) {
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj) {
                        const int j = 2 * p + jj, r = jj * 16 + (lane & 15);
                        if ((lane >> 4) == 0) {
                            const int m = m0 + wm * 128 + j * 16 + (lane & 15);
                            skey[wave][r] = epi.row(min(m, M - 1)).key;
                        }
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            uint2 h, l;
                            epi.stage2(acc[i][j], cols[i], h, l);
                            const int ch = 2 * i + ((lane >> 5) & 1);
                            // 8-B half of the 16-B chunk: flipped for rows r with bit 3 set, so the
                            // 16 rows of one b64 write group (r and r + 8 share a chunk slot under
                            // the r & 7 swizzle) fill 16 distinct 8-B banks (the LDS write rule,
                            // profiles/r05x_lds_calibration.txt); the reader swaps them back
                            const int o = r * 128 + ((ch ^ (r & 7)) << 4) + 8 * (((lane >> 4) ^ (r >> 3)) & 1);
                            *reinterpret_cast<uint2*>(img + o) = h;
                            *reinterpret_cast<uint2*>(img + 4096 + o) = l;
                        }
                    }
                    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's image written
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int it = 0; it < 8; ++it) {
                        const int L = it * 64 + lane, q = L >> 8, r = (L >> 3) & 31, ch = L & 7;
                        const int m = m0 + wm * 128 + p * 32 + r;
                        uint4 d = *reinterpret_cast<const uint4*>(img + q * 4096 + r * 128 + ((ch ^ (r & 7)) << 4));
                        if ((r >> 3) & 1) d = make_uint4(d.z, d.w, d.x, d.y);
                        if (m < M) epi.put(m, nw + ch * 8, q, skey[wave][r], d);
                    }
                    __builtin_amdgcn_s_waitcnt(0xc07f);  // image read before the next pass writes it
                    __builtin_amdgcn_wave_barrier();
                }
            } else if (m0 + TM <= M) {
                epilogue(std::false_type{});
            } else {
                epilogue(std::true_type{});
            }
            __syncthreads();  // every wave's image read: the next tile DMAs into st1
        } else if constexpr (STG == 2) {
            const int nw = n0 + wn * 64;
            char* img = st1 + wave * 8192;
            typename Epi::Col cols[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) cols[i] = epi.col(nw + i * 16 + (lane >> 4) * 4);
#pragma unroll
            for (int p = 0; p < 4; ++p) {
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    const int j = 2 * p + jj, r = jj * 16 + (lane & 15);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int ch = 4 * i + (lane >> 4);  // 16-B f32 chunk of the 256-B row
                        *reinterpret_cast<float4*>(img + r * 256 + ((ch ^ (r & 15)) << 4)) =
                            epi.stage4(acc[i][j], cols[i]);
                    }
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
                float4 xv[8];
#pragma unroll
                for (int it = 0; it < 8; ++it) {
                    const int L = it * 64 + lane, r = L >> 4, ch = L & 15;
                    xv[it] = epi.load4(mz + min(m0 + wm * 128 + p * 32 + r, M - 1), nw + ch * 4);
                }
#pragma unroll
                for (int it = 0; it < 8; ++it) {
                    const int L = it * 64 + lane, r = L >> 4, ch = L & 15;
                    const int m = m0 + wm * 128 + p * 32 + r;
                    const float4 y = *reinterpret_cast<const float4*>(img + r * 256 + ((ch ^ (r & 15)) << 4));
                    if (m < M) epi.put4(mz + m, nw + ch * 4, xv[it], y);
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
            }
            __syncthreads();  // every wave's image read: the next tile DMAs into st1
        } else {
            if (m0 + TM <= M) epilogue(std::false_type{});
            else epilogue(std::true_type{});
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) oa[i] = na[i];
        sa = nsa;
        sb = nsb;
    }
    __builtin_amdgcn_s_waitcnt(0xF70);
#undef S256_COMPUTE
#undef S256_DMA
}

// Split-bf16 GEMM, 192 x 192 form (MLG_SPLIT_TILE=192): the same three products per
// K-step of 32 as k_gemm256s on a 192 x 192 tile, whose four operand planes (48 KiB) fit a
// THREE-stage LDS-DMA ring (144 KiB): each K-step's planes are fetched two compute steps
// ahead instead of one.  The ring runs on across the workgroup's output tiles (flat step
// index over its tiles; steps past the last re-fetch the last one into a slot already
// consumed).  Same per-output MFMA order as k_gemm256s, so the same bits.
template <class Epi>
__global__ __launch_bounds__(512, 1) void k_gemm192s(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K0, int lda, int ldw, Epi epi) {
    constexpr int BK = 32, TM = 192, TN = 192;
    constexpr int PLANE = TM * BK * 2;  // 12 KiB
    constexpr int STAGE = 4 * PLANE;    // A_hi, A_lo, W_hi, W_lo
    constexpr int PIECES = 6;           // 1 KiB DMA wave-instructions per wave and stage (48 / 8 waves)
    __shared__ __attribute__((aligned(16))) char ring[3 * STAGE];
    // wave index through readfirstlane: the DMA bases derived from it stay in SGPRs
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nN = N / TN, nM = (M + TM - 1) / TM, ntiles = nN * nM;
    const int xcd = blockIdx.x & 7, per_xcd = gridDim.x >> 3;
    const int tx = (ntiles + 7) >> 3;
    const int tile_end = min((xcd + 1) * tx, ntiles);
    const int tile0 = xcd * tx + (blockIdx.x >> 3);
    if (tile0 >= tile_end) return;
    const int ntl = (tile_end - tile0 + per_xcd - 1) / per_xcd;
    const int nk = K0 / BK;
    const int S = ntl * nk;

    const int lr = lane >> 2, lp = lane & 3;
    const int wm = wave & 1, wn = wave >> 1;
    // piece i of this wave: plane pl = p / 12 (0 A_hi, 1 A_lo, 2 W_hi, 3 W_lo), rows 16 (p % 12) ..
    int prow[PIECES], pplane[PIECES];
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
        const int p = wave * PIECES + i;
        pplane[i] = p / 12;
        prow[i] = (p % 12) * 16 + lr;
    }
    auto issue = [&](int st, int slot) {  // DMA of flat step st into ring slot `slot`
        const int q = st / nk, k = st - q * nk;
        const int tile = tile0 + q * per_xcd;
        const int m0 = (tile / nN) * TM, n0 = (tile - (tile / nN) * nN) * TN;
        const unsigned b = lds_addr(ring + slot * STAGE);
#pragma unroll
        for (int i = 0; i < PIECES; ++i) {
            const int row = prow[i], pl = pplane[i];
            const int sw = (lp ^ ((row >> 1) & 3)) * 8;
            const unsigned dst = b + pl * PLANE + (row - lr) * 64;
            if (pl < 2) {
                const unsigned off = (unsigned)((min(m0 + row, M - 1) - m0) * lda + sw) * 2u;
                dma16s(off, A + (size_t)m0 * lda + k * BK + (pl ? K0 : 0), dst);
            } else {
                const unsigned off = (unsigned)(row * ldw + sw) * 2u;
                dma16s(off, W + (size_t)n0 * ldw + k * BK + (pl == 3 ? K0 : 0), dst);
            }
        }
    };
    f32x4 acc[3][6];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    issue(0, 0);
    issue(min(1, S - 1), 1);
    __builtin_amdgcn_s_waitcnt(0xF70 | PIECES);  // vmcnt(6): step 0 has landed
    __builtin_amdgcn_s_barrier();
    const int ch = lane >> 4;
    for (int st = 0; st < S; ++st) {
        issue(min(st + 2, S - 1), (st + 2) % 3);  // into the slot step st - 1 used (all waves are past it)
        const char* P = ring + (st % 3) * STAGE;
        {
            bf16x8 af[6], wh[3], wl[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int row = wn * 48 + i * 16 + (lane & 15);
                wh[i] = *reinterpret_cast<const bf16x8*>(P + 2 * PLANE + soff<32>(row, ch));
                wl[i] = *reinterpret_cast<const bf16x8*>(P + 3 * PLANE + soff<32>(row, ch));
            }
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int row = wm * 96 + j * 16 + (lane & 15);
                af[j] = *reinterpret_cast<const bf16x8*>(P + soff<32>(row, ch));
            }
#pragma unroll
            for (int j = 0; j < 6; ++j)
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[i], af[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[i], af[j], acc[i][j], 0, 0, 0);
                }
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int row = wm * 96 + j * 16 + (lane & 15);
                af[j] = *reinterpret_cast<const bf16x8*>(P + PLANE + soff<32>(row, ch));
            }
#pragma unroll
            for (int j = 0; j < 6; ++j)
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[i], af[j], acc[i][j], 0, 0, 0);
        }
        const int q = st / nk;
        if (st - q * nk == nk - 1) {  // the tile's last K-step: epilogue
            const int tile = tile0 + q * per_xcd;
            const int mt = tile / nN, m0 = mt * TM, n0 = (tile - mt * nN) * TN;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const int n = n0 + wn * 48 + i * 16 + (lane >> 4) * 4;
                    const int m = m0 + wm * 96 + j * 16 + (lane & 15);
                    if (m < M) epi(m, n, acc[i][j]);
                    acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0): stores counted there too
        } else {
            __builtin_amdgcn_s_waitcnt(0xF70 | PIECES);  // vmcnt(6): step st + 1 has landed
        }
        __builtin_amdgcn_s_barrier();
    }
    __builtin_amdgcn_s_waitcnt(0xF70);
}

// Variant 5: the 256 x 256 persistent tile of k_gemm256 with K-tiles of 32 in a 4-deep
// LDS ring (4 x 32 KiB): the DMA of K-tile t + 3 is issued when t is computed, so three
// compute steps (not one) hide each tile's fetch; the ring runs on across output tiles
// (the last three steps of a tile fetch the next tile's first three K-tiles).  Same MFMA
// k order as k_gemm256, so the same bits.
template <class Epi>
__global__ __launch_bounds__(512, 2) void k_gemm256q(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                    int M, int N, int K, int lda, int ldw, Epi epi) {
    constexpr int BK = 32, TM = 256, TN = 256;
    constexpr int A_BYTES = TM * BK * 2, STAGE = (TM + TN) * BK * 2;  // 32 KiB
    constexpr int NA = 2, NB = 2;                                      // DMAs per wave per K-tile
    constexpr int WAIT2 = 0xF70 | (2 * (NA + NB));                     // two newer K-tiles may fly
    __shared__ __attribute__((aligned(16))) char ringbuf[4 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nN = N / TN, nM = (M + TM - 1) / TM, ntiles = nN * nM;
    const int xcd = blockIdx.x & 7, per_xcd = gridDim.x >> 3;
    const int tx = (ntiles + 7) >> 3;
    const int tile_end = min((xcd + 1) * tx, ntiles);
    int tile = xcd * tx + (blockIdx.x >> 3);
    if (tile >= tile_end) return;

    const int lr = lane >> 2, lp = lane & 3;  // 16 rows x 4 chunks of 16 B per DMA wave-instruction
    const int wm = wave & 1, wn = wave >> 1;
    const int da = NA * wave * 1024, db = A_BYTES + NB * wave * 1024;
    const int nk = K / BK;  // >= 3 (checked by the launcher)
    unsigned ob[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int row = (NB * wave + i) * 16 + lr;
        ob[i] = (unsigned)(row * ldw + ((lp ^ ((row >> 1) & 3)) * 8)) * 2u;
    }
    auto a_offsets = [&](int t, unsigned* oa) {
        const int m0 = (t / nN) * TM;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int row = (NA * wave + i) * 16 + lr;
            oa[i] = (unsigned)((min(m0 + row, M - 1) - m0) * lda + ((lp ^ ((row >> 1) & 3)) * 8)) * 2u;
        }
    };
    auto a_base = [&](int t) { return A + (size_t)((t / nN) * TM) * lda; };
    auto b_base = [&](int t) { return W + (size_t)((t % nN) * TN) * ldw; };
#define Q256_DMA(ST, OA, SA, SB, k0)                                                                       \
    {                                                                                                      \
        const unsigned b_ = lds_addr(ST);                                                                  \
        const bf16_t* sa_ = (SA) + (k0);                                                                   \
        const bf16_t* sb_ = (SB) + (k0);                                                                   \
        _Pragma("unroll") for (int i = 0; i < NA; ++i) dma16s((OA)[i], sa_, b_ + da + i * 1024);           \
        _Pragma("unroll") for (int i = 0; i < NB; ++i) dma16s(ob[i], sb_, b_ + db + i * 1024);             \
    }
    // the K-tile stream: (tile, k) pairs in order, the fetch position runs 3 ahead
    int ftile = tile, fk = 0;
    unsigned foa[NA];
    a_offsets(ftile, foa);
    const bf16_t* fsa = a_base(ftile);
    const bf16_t* fsb = b_base(ftile);
    int fslot = 0;
    auto fetch_next = [&]() {
        Q256_DMA(ringbuf + fslot * STAGE, foa, fsa, fsb, fk * BK);
        fslot = (fslot + 1) & 3;
        if (++fk == nk) {  // continue with the next output tile of this workgroup (or re-read)
            fk = 0;
            if (ftile + per_xcd < tile_end) {
                ftile += per_xcd;
                a_offsets(ftile, foa);
                fsa = a_base(ftile);
                fsb = b_base(ftile);
            } else {
                fk = nk - 1;  // past the last tile: harmless re-reads of its last K-tile
            }
        }
    };
    fetch_next();
    fetch_next();
    fetch_next();
    __builtin_amdgcn_s_waitcnt(WAIT2);
    __builtin_amdgcn_s_barrier();
    int cslot = 0;
    for (; tile < tile_end; tile += per_xcd) {
        f32x4 acc[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < nk; ++t) {
            fetch_next();  // K-tile t + 3 of the stream, into the slot computed last step
            const char* ST = ringbuf + cslot * STAGE;
            bf16x8 af[8], wf[4];
            const int ch = lane >> 4;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = wn * 64 + i * 16 + (lane & 15);
                wf[i] = *reinterpret_cast<const bf16x8*>(ST + A_BYTES + soff<32>(row, ch));
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int row = wm * 128 + j * 16 + (lane & 15);
                af[j] = *reinterpret_cast<const bf16x8*>(ST + soff<32>(row, ch));
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);
            cslot = (cslot + 1) & 3;
            __builtin_amdgcn_s_waitcnt(WAIT2);  // K-tile t + 1 has landed (t + 2, t + 3 may fly)
            __builtin_amdgcn_s_barrier();
        }
        const int mt = tile / nN, m0 = mt * TM, n0 = (tile - mt * nN) * TN;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4;
                const int m = m0 + wm * 128 + j * 16 + (lane & 15);
                if (m < M) epi(m, n, acc[i][j]);
            }
    }
    __builtin_amdgcn_s_waitcnt(0xF70);
#undef Q256_DMA
}
// Implicit-GEMM convolution on the persistent 256 x TN x 64 tile of k_gemm256 (LoFTR's
// ResNetFPN, loftr.hip): A[m, k] is never materialised.  Row m = output pixel (b, oy, ox)
// of an NHWC bf16 input [B, H, W, C]; k = tap * C + c with C % 64 == 0, so a 64-wide
// K-tile lies inside one tap (ty, tx) and its 16-B chunks are contiguous input channels
// at pixel (oy * s - pad + ty, ox * s - pad + tx).  Each lane keeps its 4 rows' pixel
// origin per output tile and LDS-DMAs from a per-lane 64-bit address; taps that fall in
// the zero padding read a 16-B zero line (`zero`).  TN = 256: 8 waves 2 (M) x 4 (N) of
// 128 x 64; TN = 128: 4 (M) x 2 (N) of 64 x 64.  Same MFMA k order as the explicit
// im2col GEMM, so the same bits.
#ifndef MLG_CONV_STAGED
#define MLG_CONV_STAGED 1
#endif
struct ConvGeom {
    const bf16_t* in; const bf16_t* zero; int H, W, C, kw, s, pad, Ho, Wo;
};

template <class Epi, int TN>
__global__ __launch_bounds__(512, 2) void k_conv256(ConvGeom g, const bf16_t* __restrict__ W, int M, int N, int K,
                                                    Epi epi) {
    constexpr int BK = 64, TM = 256;
    constexpr int WN = TN / 64, WM = 8 / WN, RM = TM / WM;  // waves along N / M, rows per wave
    constexpr int JM = RM / 16;                             // 16-row m-tiles per wave
    constexpr int A_BYTES = TM * BK * 2, STAGE = (TM + TN) * BK * 2;
    constexpr int NA = 4, NB = TN / 64;  // DMAs per wave per K-tile
    __shared__ __attribute__((aligned(16))) char st0[STAGE];
    __shared__ __attribute__((aligned(16))) char st1[STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nN = N / TN, nM = (M + TM - 1) / TM, ntiles = nN * nM;
    const int xcd = blockIdx.x & 7, per_xcd = gridDim.x >> 3;
    const int tx = (ntiles + 7) >> 3;
    const int tile_end = min((xcd + 1) * tx, ntiles);
    int tile = xcd * tx + (blockIdx.x >> 3);
    if (tile >= tile_end) return;

    const int lr = lane >> 3, lp = lane & 7;
    const int wm = wave % WM, wn = wave / WM;
    const int da = NA * wave * 1024, db = A_BYTES + NB * wave * 1024;
    const int nk = K / BK;  // even (checked by the launcher)

    unsigned ob[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int row = (NB * wave + i) * 8 + lr;
        ob[i] = (unsigned)(row * K + ((lp ^ ((row >> 1) & 7)) * 8)) * 2u;
    }
    // per row: (b, oy, ox) packed 10 / 11 / 11 bits (H, W <= 2048 and B <= 1024, checked
    // by the launcher) -- one VGPR per row instead of three
    unsigned pk[NA];
    auto rows_of = [&](int t) {
        const int m0 = (t / nN) * TM;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int row = (NA * wave + i) * 8 + lr;
            const int m = min(m0 + row, M - 1);
            const int ox = m % g.Wo, r = m / g.Wo, oy = r % g.Ho, b = r / g.Ho;
            pk[i] = ((unsigned)b << 22) | ((unsigned)oy << 11) | (unsigned)ox;
        }
    };
    auto a_src = [&](int i, int k0) -> const bf16_t* {
        const int tap = k0 / g.C, c0 = k0 - tap * g.C;
        const int ty = tap / g.kw, tx_ = tap - ty * g.kw;
        const int b = (int)(pk[i] >> 22), oy = (int)((pk[i] >> 11) & 2047u), ox = (int)(pk[i] & 2047u);
        const int iy = oy * g.s - g.pad + ty, ix = ox * g.s - g.pad + tx_;
        const int row = (NA * wave + i) * 8 + lr;
        const int ch = (lp ^ ((row >> 1) & 7)) * 8;
        if ((unsigned)iy >= (unsigned)g.H || (unsigned)ix >= (unsigned)g.W) return g.zero;
        return g.in + ((size_t)((b * g.H + iy) * g.W + ix)) * g.C + c0 + ch;
    };
    auto b_base = [&](int t) { return W + (size_t)((t % nN) * TN) * K; };
    const bf16_t* sb = b_base(tile);
    rows_of(tile);
#define C256_DMA(ST, SB, k0)                                                                               \
    {                                                                                                      \
        const unsigned b_ = lds_addr(ST);                                                                  \
        const bf16_t* sb_ = (SB) + (k0);                                                                   \
        _Pragma("unroll") for (int i = 0; i < NA; ++i) dma16(a_src(i, k0), b_ + da + i * 1024);            \
        _Pragma("unroll") for (int i = 0; i < NB; ++i) dma16s(ob[i], sb_, b_ + db + i * 1024);             \
    }
#define C256_COMPUTE(ST)                                                                                   \
    _Pragma("unroll") for (int s = 0; s < 2; ++s) {                                                        \
        bf16x8 af[JM], wf[4];                                                                              \
        const int ch = s * 4 + (lane >> 4);                                                                \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                    \
            const int row = wn * 64 + i * 16 + (lane & 15);                                                \
            wf[i] = *reinterpret_cast<const bf16x8*>((ST) + A_BYTES + soff<64>(row, ch));                  \
        }                                                                                                  \
        _Pragma("unroll") for (int j = 0; j < JM; ++j) {                                                   \
            const int row = wm * RM + j * 16 + (lane & 15);                                                \
            af[j] = *reinterpret_cast<const bf16x8*>((ST) + soff<64>(row, ch));                            \
        }                                                                                                  \
        _Pragma("unroll") for (int j = 0; j < JM; ++j) _Pragma("unroll") for (int i = 0; i < 4; ++i)       \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);         \
    }

    C256_DMA(st0, sb, 0);
    __builtin_amdgcn_s_waitcnt(0xF70);
    __builtin_amdgcn_s_barrier();
    for (; tile < tile_end; tile += per_xcd) {
        const int next = tile + per_xcd < tile_end ? tile + per_xcd : tile;
        const bf16_t* nsb = b_base(next);
        const int kn = next != tile ? 0 : nk - 1;  // K-tile of the last DMA (no next tile: harmless re-read)
        f32x4 acc[4][JM];  // [n-tile][m-tile]
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < JM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < nk; t += 2) {
            C256_DMA(st1, sb, (t + 1) * BK);
            C256_COMPUTE(st0);
            __builtin_amdgcn_s_waitcnt(0xF70);
            __builtin_amdgcn_s_barrier();
            if (t + 2 < nk) {
                C256_DMA(st0, sb, (t + 2) * BK);
            } else {
                rows_of(next);  // this tile's A rows are no longer needed
                C256_DMA(st0, nsb, kn);     // K-tile 0 of the next output tile
            }
            C256_COMPUTE(st1);
            __builtin_amdgcn_s_waitcnt(0xF70);
            __builtin_amdgcn_s_barrier();
        }
        const int mt = tile / nN, m0 = mt * TM, n0 = (tile - mt * nN) * TN;
        if constexpr (MLG_CONV_STAGED) {
            // row-staged (gemm256_rows_epilogue; timing probe with the epilogue skipped: the
            // LoFTR backbone 29 % faster, the staged form -3 %, profiles/
            // r06r_ab_conv_staged_epilogue.txt)
            gemm256_rows_epilogue<RM, STAGE / 8>(epi, acc, st1 + wave * (STAGE / 8), m0 + wm * RM, n0 + wn * 64, M,
                                                 lane);
            __syncthreads();  // every wave's image read: the next tile DMAs into st1
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < JM; ++j) {
                    const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4;
                    const int m = m0 + wm * RM + j * 16 + (lane & 15);
                    if (m < M) epi(m, n, acc[i][j]);
                }
        }
        sb = nsb;
    }
    __builtin_amdgcn_s_waitcnt(0xF70);
#undef C256_COMPUTE
#undef C256_DMA
}
}  // namespace dma

// 1: 128x128 register-staged; 2: 128x256 DMA BK=64 (3 stages); 3: 128x256 DMA BK=32 (2 WG/CU);
// 4: persistent 256x256 DMA where N allows (N % 256 == 0, K / 64 even), else 2.
// Fixed per build (MLG_GEMM_VARIANT; A/B arms are separate builds loaded through
// tools/ab_run.py) or per process through mlg_gemm_set_variant (tools/gemm_bench.py).
#ifndef MLG_GEMM_VARIANT
#define MLG_GEMM_VARIANT 4
#endif
int g_variant = MLG_GEMM_VARIANT;
int g_num_cus = 256;  // multiple of 8 (refreshed from the device on first use)

int num_cus() {
    static int cached = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount,
                                                                         dev) != hipSuccess || n < 8)
            return 256;
        return n / 8 * 8;
    }();
    return cached;
}

template <class Epi>
int launch(const bf16_t* A, const bf16_t* W, int M, int N, int K, int lda, int ldw, Epi epi, hipStream_t s,
           int variant = -1) {
    if (variant < 0) variant = g_variant;
    g_num_cus = num_cus();
    if (M <= 0 || N <= 0 || K <= 0 || (K % BK) || (lda % 8) || (ldw % 8) || lda < K || ldw < K)
        return MLG_EINVAL;
    if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W)) & 15) return MLG_EINVAL;
    const long nwg_dma = (long)(N / dma::BN) * ((M + dma::BM - 1) / dma::BM);
    if (variant == 5 && N % 256 == 0 && K % 32 == 0 && K / 32 >= 3) {
        const long ntiles = (long)(N / 256) * ((M + 255) / 256);
        const long grid = std::min<long>(g_num_cus, (ntiles + 7) / 8 * 8);  // persistent: <= 1 per CU
        hipLaunchKernelGGL(dma::k_gemm256q<Epi>, dim3((unsigned)grid), dim3(512), 0, s, A, W, M, N, K, lda, ldw, epi);
    } else if ((variant == 4 || variant == 5) && N % 256 == 0 && (K / 64) % 2 == 0) {
        const long ntiles = (long)(N / 256) * ((M + 255) / 256);
        const long grid = std::min<long>(g_num_cus, (ntiles + 7) / 8 * 8);  // persistent: <= 1 per CU
        hipLaunchKernelGGL(dma::k_gemm256<Epi>, dim3((unsigned)grid), dim3(512), 0, s, A, W, M, N, K, lda, ldw, epi);
    } else if (variant == 3 && N % dma::BN == 0 && (K / 32) % 3 == 0) {
        hipLaunchKernelGGL((dma::k_gemm<Epi, 32>), dim3((unsigned)nwg_dma), dim3(512), 0, s, A, W, M, N, K, lda, ldw,
                           epi);
    } else if (variant >= 2 && N % dma::BN == 0 && (K / 64) % 3 == 0) {
        hipLaunchKernelGGL((dma::k_gemm<Epi, 64>), dim3((unsigned)nwg_dma), dim3(512), 0, s, A, W, M, N, K, lda, ldw,
                           epi);
    } else {
        if (N % BN) return MLG_EINVAL;
        const long nwg = (long)(N / BN) * ((M + BM - 1) / BM);
        hipLaunchKernelGGL(k_gemm_nt<Epi>, dim3((unsigned)nwg), dim3(256), 0, s, A, W, M, N, K, lda, ldw, epi);
    }
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

// Split-bf16 GEMM (MLG_VIT_SPLIT): A rows [A_hi | A_lo] of K0 each (lda >= 2 K0), W rows
// [W_hi | W_lo] (ldw >= 2 K0); dma::k_gemm256s
template <class Epi>
#ifndef MLG_SPLIT_TILE
#define MLG_SPLIT_TILE 256
#endif
int launch_split(const bf16_t* A, const bf16_t* W, int M, int N, int K0, int lda, int ldw, Epi epi, hipStream_t s,
                 int nb = 1, long sA = 0, long sW = 0) {
    g_num_cus = num_cus();
    if (M <= 0 || K0 <= 0 || K0 % 64 || lda < 2 * K0 || ldw < 2 * K0 || (lda % 8) || (ldw % 8)) return MLG_EINVAL;
    if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W)) & 15) return MLG_EINVAL;
    // batched products: staged-f32 epilogues only (their row index is the only per-problem
    // output coordinate), 16-B aligned problem bases
    if (nb < 1 || (nb > 1 && (dma::staged_of<Epi>::value != 2 || ((sA | sW) & 7)))) return MLG_EINVAL;
    if (MLG_SPLIT_TILE == 192 && N % 192 == 0 && nb == 1) {
        const long nt = (long)(N / 192) * ((M + 191) / 192);
        const long g = std::min<long>(g_num_cus, (nt + 7) / 8 * 8);
        hipLaunchKernelGGL(dma::k_gemm192s<Epi>, dim3((unsigned)g), dim3(512), 0, s, A, W, M, N, K0, lda, ldw, epi);
        MLG_LAUNCH_CHECK();
        return MLG_OK;
    }
    if (N % 256) return MLG_EINVAL;
    const long ntiles = (long)nb * (N / 256) * ((M + 255) / 256);
    if (ntiles > INT32_MAX) return MLG_EINVAL;
    const long grid = std::min<long>(g_num_cus, (ntiles + 7) / 8 * 8);
    hipLaunchKernelGGL(dma::k_gemm256s<Epi>, dim3((unsigned)grid), dim3(512), 0, s, A, W, M, N, K0, lda, ldw, epi, nb,
                       sA, sW);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

}  // namespace

int mlg_gemm_qkv_split(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* Q, bf16_t* Kh, bf16_t* V, int M,
                       int T, int Tpad, size_t lo_off, hipStream_t s) {
    if (M % T) return MLG_EINVAL;
    return launch_split(A, W, M, 3 * 768, 768, 2 * 768, 2 * 768,
                        EpiQKVSplit{Q, Kh, V, bias, T, Tpad, (M / T) * Tpad, lo_off}, s);
}
int mlg_gemm_residual_split(const bf16_t* A, const bf16_t* W, const float* bias, const float* gamma, float* X, int M,
                            int N, int K0, hipStream_t s) {
    return launch_split(A, W, M, N, K0, 2 * K0, 2 * K0, EpiResidual{X, N, bias, gamma}, s);
}
int mlg_gemm_bias_gelu_split(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* C, int M, int N, int K0,
                             hipStream_t s) {
    return launch_split(A, W, M, N, K0, 2 * K0, 2 * K0, EpiBiasGeluSplit{C, 2 * N, N, bias}, s);
}
int mlg_gemm_patch_split(const bf16_t* A, const bf16_t* W, const float* bias, const float* pos, float* X, int M, int P,
                         int Kpad, hipStream_t s) {
    if (M % P) return MLG_EINVAL;
    return launch_split(A, W, M, 768, Kpad, 2 * Kpad, 2 * Kpad, EpiPatch{X, bias, pos, P}, s);
}

int mlg_gemm_sim_split_loftr(const bf16_t* A, const bf16_t* B, int M, int Npad, int K0, float* S, int lds, int ncols,
                             hipStream_t s, int nb, long pstride) {
    if (ncols > Npad || ncols > lds || lds > Npad || (lds % 4)) return MLG_EINVAL;
    return launch_split(A, B, M, Npad, K0, 2 * K0, 2 * K0, EpiSimLoFTR{S, lds, ncols}, s, nb, pstride, pstride);
}

int mlg_gemm_f32out(const bf16_t* A, const bf16_t* W, float* C, int M, int N, int K, hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiF32{C, N}, s);
}
int mlg_gemm_f32out_variant(int variant, const bf16_t* A, const bf16_t* W, float* C, int M, int N, int K,
                            hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiF32{C, N}, s, variant);
}
int mlg_gemm_bias_f32_ld(const bf16_t* A, int lda, const bf16_t* W, const float* bias, float* C, int ldc, int M,
                         int N, int K, hipStream_t s) {
    return launch(A, W, M, N, K, lda, K, EpiBiasF32{C, ldc, bias}, s);
}
int mlg_gemm_bias_split_bf16(const bf16_t* A, int lda, const bf16_t* W, const float* bias, bf16_t* H, bf16_t* L,
                             int M, int N, int K, hipStream_t s) {
    if (N % 16) return MLG_EINVAL;
    return launch(A, W, M, N, K, lda, K, EpiBiasSplitBF16{H, L, M, bias}, s);
}
int mlg_gemm_bias_relu_bf16(const bf16_t* A, int lda, const bf16_t* W, const float* bias, bf16_t* C, int ldc,
                            int nvalid, int M, int N, int K_, hipStream_t s) {
    return launch(A, W, M, N, K_, lda, K_, EpiBiasReluBF16{C, ldc, bias, nvalid}, s);
}
int mlg_gemm_bias_add_relu(const bf16_t* A, int lda, const bf16_t* W, const float* bias, const float* R, float* X,
                           int ldx, bf16_t* C, int M, int N, int K_, hipStream_t s) {
    return launch(A, W, M, N, K_, lda, K_, EpiBiasAddRelu{R, X, ldx, C, bias}, s);
}
int mlg_gemm_conv(const bf16_t* A, int lda, const bf16_t* W, const float* bias, const float* R, int ldr, float* X,
                  int ldx, bf16_t* C, int ldc, int act, int act_cols, int M, int N, int K_, hipStream_t s, float vdiv) {
    if ((!X && !C) || act < 0 || act > 3) return MLG_EINVAL;
    return launch(A, W, M, N, K_, lda, K_, EpiConv{bias, R, ldr, X, ldx, C, ldc, act, act_cols, vdiv}, s);
}
int mlg_gemm_conv_upadd(const bf16_t* A, int lda, const bf16_t* W, const float* bias, const float* src, int h, int w,
                        bf16_t* C, int M, int N, int K_, hipStream_t s) {
    if (!src || !C || h < 1 || w < 1 || (N % 4) || M % (4 * h * w)) return MLG_EINVAL;
    return launch(A, W, M, N, K_, lda, K_, EpiConvUp{bias, src, h, w, C, N}, s);
}
int mlg_gemm_set_variant(int variant) {
    if (variant < 1 || variant > 5) return MLG_EINVAL;
    g_variant = variant;
    return MLG_OK;
}
int mlg_gemm_bias_bf16(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* C, int M, int N, int K,
                       hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiBiasBF16{C, N, bias}, s);
}
int mlg_gemm_bias_gelu_bf16(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* C, int M, int N, int K,
                            hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiBiasGeluBF16{C, N, bias}, s);
}
int mlg_gemm_residual(const bf16_t* A, const bf16_t* W, const float* bias, const float* gamma, float* X, int M,
                      int N, int K, hipStream_t s) {
    return launch(A, W, M, N, K, K, K, EpiResidual{X, N, bias, gamma}, s);
}
int mlg_gemm_qkv(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* Q, bf16_t* Kh, bf16_t* V, int M,
                 int T, int Tpad, hipStream_t s) {
    if (M % T || Tpad % 64 || Tpad < T) return MLG_EINVAL;
    return launch(A, W, M, 3 * 768, 768, 768, 768, EpiQKV{Q, Kh, V, bias, T, Tpad, (M / T) * Tpad}, s);
}
int mlg_gemm_patch(const bf16_t* A, const bf16_t* W, const float* bias, const float* pos, float* X, int M, int P,
                   int Kpad, hipStream_t s) {
    if (M % P) return MLG_EINVAL;
    return launch(A, W, M, 768, Kpad, Kpad, Kpad, EpiPatch{X, bias, pos, P}, s);
}
int mlg_conv_implicit(const bf16_t* in, const bf16_t* zero, int B, int H, int W, int C, int k, int s,
                      const bf16_t* Wt, const float* bias, const float* R, int ldr, float* X, int ldx, bf16_t* Cout,
                      int ldc, int act, int act_cols, int N, hipStream_t st) {
    if ((!X && !Cout) || act < 0 || act > 3 || !in || !zero || !Wt || B <= 0 || H <= 0 || W <= 0 || C % 64 ||
        (k != 1 && k != 3) || s < 1 || N <= 0 || N % 128)
        return MLG_EINVAL;
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(zero) | reinterpret_cast<uintptr_t>(Wt)) & 15)
        return MLG_EINVAL;
    const int Ho = (H + s - 1) / s, Wo = (W + s - 1) / s, K = k * k * C;
    if ((K / 64) % 2 || B > 1024 || H > 2048 || W > 2048 || (long)B * H * W >= (1L << 31)) return MLG_EINVAL;
    const int M = B * Ho * Wo;
    const dma::ConvGeom g{in, zero, H, W, C, k, s, k / 2, Ho, Wo};
    const EpiConv epi{bias, R, ldr, X, ldx, Cout, ldc, act, act_cols};
    const int cus = num_cus();
    if (N % 256 == 0) {
        const long ntiles = (long)(N / 256) * ((M + 255) / 256);
        const long grid = std::min<long>(cus, (ntiles + 7) / 8 * 8);
        hipLaunchKernelGGL((dma::k_conv256<EpiConv, 256>), dim3((unsigned)grid), dim3(512), 0, st, g, Wt, M, N, K, epi);
    } else {
        const long ntiles = (long)(N / 128) * ((M + 255) / 256);
        const long grid = std::min<long>(cus, (ntiles + 7) / 8 * 8);
        hipLaunchKernelGGL((dma::k_conv256<EpiConv, 128>), dim3((unsigned)grid), dim3(512), 0, st, g, Wt, M, N, K, epi);
    }
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}
