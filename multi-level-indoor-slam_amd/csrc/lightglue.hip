// LightGlue matcher for a batch of keyframe pairs (gfx950).
//
// Restates LightGlue(features='superpoint') as called by the reference
// (geometric_verification.py:224-233, 285-305; semantics in oracle/lightglue.py).
// All images of all pairs live in ONE flat token layout: segment 2p (image a of pair
// p) and 2p+1 (image b), each padded to a multiple of 64 rows.  Per layer the shared
// weights run as single GEMMs over every token (gemm_bf16.hip, bf16 MFMA, f32
// accumulation); attention is one ragged launch (attention.hip k_attention_varlen)
// whose tasks are the self (seg -> seg) or cross (a -> b, b -> a) pairings.
// State: x f32 [Npad, 256] (residual stream) and cat bf16 [Npad, 512] = [x | message]
// so the FFN's torch.cat([x, message]) is free.  After each layer but the last the
// token confidences and matchability give per-segment statistics; the host reads them
// (one small D2H copy per layer), stops pairs whose confident ratio exceeds
// depth_confidence (their assignment runs at that layer), prunes segments above the
// pruning threshold, and compacts the layout with one gather.
#include <vector>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int LG_D = 256, LG_H = 4, LG_L = 9;

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float logsigmoidf(float x) {
    // log(sigmoid(x)) = min(x, 0) - log1p(exp(-|x|))  (torch's stable form)
    return fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
}

struct Seg {
    int off, len, frame, pad;  // flat row offset, live tokens, source frame, unused
};

// ------------------------------------------------------------------ init
// One workgroup per segment: normalize_keypoints (size = 1 + max - min), Fourier
// positional encoding (cos / sin of Wr . k, 32 frequencies), x = desc, cat[:, :256] =
// bf16(desc), ind = source index; rows past len zeroed.
__global__ __launch_bounds__(256) void k_lg_init(const Seg* __restrict__ segs, const float* __restrict__ kpts,
                                                 const float* __restrict__ desc, int kmax,
                                                 const float* __restrict__ Wr, float* __restrict__ x,
                                                 bf16_t* __restrict__ cat, float* __restrict__ ecos,
                                                 float* __restrict__ esin, int32_t* __restrict__ ind) {
    const Seg sg = segs[blockIdx.x];
    const int tid = threadIdx.x;
    const float* kp = kpts + (size_t)sg.frame * kmax * 2;
    const float* ds = desc + (size_t)sg.frame * kmax * LG_D;
    __shared__ float red[4][256];
    float mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
    for (int i = tid; i < sg.len; i += 256) {
        mnx = fminf(mnx, kp[2 * i]); mxx = fmaxf(mxx, kp[2 * i]);
        mny = fminf(mny, kp[2 * i + 1]); mxy = fmaxf(mxy, kp[2 * i + 1]);
    }
    red[0][tid] = mnx; red[1][tid] = mny; red[2][tid] = mxx; red[3][tid] = mxy;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) {
            red[0][tid] = fminf(red[0][tid], red[0][tid + o]);
            red[1][tid] = fminf(red[1][tid], red[1][tid + o]);
            red[2][tid] = fmaxf(red[2][tid], red[2][tid + o]);
            red[3][tid] = fmaxf(red[3][tid], red[3][tid + o]);
        }
        __syncthreads();
    }
    const float sx = 1.f + red[2][0] - red[0][0], sy = 1.f + red[3][0] - red[1][0];
    const float shx = sx / 2.f, shy = sy / 2.f, scale = fmaxf(sx, sy) / 2.f;
    const int padded = (sg.len + 63) & ~63;
    for (int i = tid; i < padded; i += 256) {
        const size_t r = (size_t)sg.off + i;
        const bool live = i < sg.len;
        float kx = 0.f, ky = 0.f;
        if (live) {
            kx = (kp[2 * i] - shx) / scale;
            ky = (kp[2 * i + 1] - shy) / scale;
        }
        for (int f = 0; f < 32; ++f) {
            const float pr = live ? kx * Wr[2 * f] + ky * Wr[2 * f + 1] : 0.f;
            ecos[r * 32 + f] = live ? cosf(pr) : 0.f;
            esin[r * 32 + f] = live ? sinf(pr) : 0.f;
        }
        ind[r] = live ? i : -1;
    }
    for (int e = tid; e < padded * LG_D; e += 256) {
        const int i = e / LG_D, c = e % LG_D;
        const size_t r = (size_t)sg.off + i;
        const float v = i < sg.len ? ds[(size_t)i * LG_D + c] : 0.f;
        x[r * LG_D + c] = v;
        cat[r * 512 + c] = f32_to_bf16(v);
    }
}

// ------------------------------------------------------------------ head rearrangement
// self: qkv f32 [Npad, 768] laid out (head, 64, 3) -> rotary q, k -> Q, K [4][Npad][64],
// V^T [4][64][Npad] (bf16); rows outside any segment's live range are zeroed.
__global__ __launch_bounds__(256) void k_lg_heads_self(const float* __restrict__ qkv, const float* __restrict__ ecos,
                                                       const float* __restrict__ esin, const uint8_t* __restrict__ live,
                                                       int Npad, bf16_t* __restrict__ Q, bf16_t* __restrict__ K,
                                                       bf16_t* __restrict__ Vt) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (row, head, pair of dims)
    if (e >= (long)Npad * LG_H * 32) return;
    const int r = (int)(e / (LG_H * 32)), h = (int)((e / 32) % LG_H), j = (int)(e % 32);
    const bool on = live[r];
    const float* b = qkv + (size_t)r * 768 + h * 192;
    const int d0 = 2 * j, d1 = 2 * j + 1;
    float q0 = b[d0 * 3 + 0], q1 = b[d1 * 3 + 0];
    float k0 = b[d0 * 3 + 1], k1 = b[d1 * 3 + 1];
    const float v0 = b[d0 * 3 + 2], v1 = b[d1 * 3 + 2];
    const float c = ecos[(size_t)r * 32 + j], s = esin[(size_t)r * 32 + j];
    // t * cos + rotate_half(t) * sin; rotate_half(t)[2j] = -t[2j+1], [2j+1] = t[2j]
    const float rq0 = q0 * c + (-q1) * s, rq1 = q1 * c + q0 * s;
    const float rk0 = k0 * c + (-k1) * s, rk1 = k1 * c + k0 * s;
    const size_t qi = ((size_t)h * Npad + r) * 64 + d0;
    *reinterpret_cast<uint32_t*>(Q + qi) = on ? pack_bf16x2(rq0, rq1) : 0u;
    *reinterpret_cast<uint32_t*>(K + qi) = on ? pack_bf16x2(rk0, rk1) : 0u;
    Vt[((size_t)h * 64 + d0) * Npad + r] = on ? f32_to_bf16(v0) : (bf16_t)0;
    Vt[((size_t)h * 64 + d1) * Npad + r] = on ? f32_to_bf16(v1) : (bf16_t)0;
}

// cross: qkv f32 [Npad, 512] = [to_qk | to_v] -> Q = K = qk heads, V^T = v heads
__global__ __launch_bounds__(256) void k_lg_heads_cross(const float* __restrict__ qkv, const uint8_t* __restrict__ live,
                                                        int Npad, bf16_t* __restrict__ Q, bf16_t* __restrict__ Vt) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (row, head, pair of dims)
    if (e >= (long)Npad * LG_H * 32) return;
    const int r = (int)(e / (LG_H * 32)), h = (int)((e / 32) % LG_H), j = (int)(e % 32);
    const bool on = live[r];
    const float* b = qkv + (size_t)r * 512;
    const int d0 = 2 * j;
    const size_t qi = ((size_t)h * Npad + r) * 64 + d0;
    *reinterpret_cast<uint32_t*>(Q + qi) = on ? pack_bf16x2(b[h * 64 + d0], b[h * 64 + d0 + 1]) : 0u;
    Vt[((size_t)h * 64 + d0) * Npad + r] = on ? f32_to_bf16(b[256 + h * 64 + d0]) : (bf16_t)0;
    Vt[((size_t)h * 64 + d0 + 1) * Npad + r] = on ? f32_to_bf16(b[256 + h * 64 + d0 + 1]) : (bf16_t)0;
}

// ------------------------------------------------------------------ FFN middle
// h = GELU(LayerNorm_512(h_f32)) -> bf16; one wave per row (8 values per lane).
__global__ __launch_bounds__(256) void k_lg_ln_gelu(const float* __restrict__ hf, const float* __restrict__ g,
                                                    const float* __restrict__ b, bf16_t* __restrict__ hb, int M) {
    const int lane = threadIdx.x & 63;
    const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= M) return;
    const float* x = hf + r * 512;
    float v[8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = x[lane + 64 * i];
        s += v[i];
    }
    const float mean = wave_sum(s) / 512.f;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float d = v[i] - mean;
        q += d * d;
    }
    const float rstd = rsqrtf(wave_sum(q) / 512.f + 1e-5f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int c = lane + 64 * i;
        const float y = (v[i] - mean) * rstd * g[c] + b[c];
        hb[r * 512 + c] = f32_to_bf16(0.5f * y * (1.f + erff(y * 0.70710678118654752f)));
    }
}

// cat[:, :256] = bf16(x)
__global__ void k_lg_sync(const float* __restrict__ x, bf16_t* __restrict__ cat, long n) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const long r = e / LG_D, c = e % LG_D;
    cat[r * 512 + c] = f32_to_bf16(x[e]);
}

// ------------------------------------------------------------------ confidences
// One workgroup per segment, one wave per token: conf = sigmoid(x . wc + bc),
// z = x . wm + bm.  stats[seg] = {#(conf < thr), #keep} with keep = sigmoid(z) > 1 - wc
// or conf <= thr (only meaningful when the segment is pruned).
__global__ __launch_bounds__(256) void k_lg_conf(const Seg* __restrict__ segs, const float* __restrict__ x,
                                                 const float* __restrict__ wc, const float* __restrict__ bc,
                                                 const float* __restrict__ wm, const float* __restrict__ bm,
                                                 float thr, float width_conf, float* __restrict__ z,
                                                 uint8_t* __restrict__ keep, int* __restrict__ stats) {
    const Seg sg = segs[blockIdx.x];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ int cnt[2];
    if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
    __syncthreads();
    int low = 0, kp = 0;
    for (int i = wave; i < sg.len; i += 4) {
        const float* xr = x + (size_t)(sg.off + i) * LG_D;
        float a = 0.f, m = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float v = xr[lane + 64 * j];
            a += v * wc[lane + 64 * j];
            m += v * wm[lane + 64 * j];
        }
        a = wave_sum(a) + bc[0];
        m = wave_sum(m) + bm[0];
        if (lane == 0) {
            const float conf = sigmoidf(a);
            const bool k = sigmoidf(m) > 1.f - width_conf || conf <= thr;
            z[sg.off + i] = m;
            keep[sg.off + i] = k;
            low += conf < thr;
            kp += k;
        }
    }
    if (lane == 0) {
        atomicAdd(&cnt[0], low);
        atomicAdd(&cnt[1], kp);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        stats[2 * blockIdx.x] = cnt[0];
        stats[2 * blockIdx.x + 1] = cnt[1];
    }
}

// z = x . wm + bm for every live token of the given segments (last-layer assignment)
__global__ __launch_bounds__(256) void k_lg_matchability(const Seg* __restrict__ segs, const float* __restrict__ x,
                                                         const float* __restrict__ wm, const float* __restrict__ bm,
                                                         float* __restrict__ z) {
    const Seg sg = segs[blockIdx.x];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = wave; i < sg.len; i += 4) {
        const float* xr = x + (size_t)(sg.off + i) * LG_D;
        float m = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) m += xr[lane + 64 * j] * wm[lane + 64 * j];
        m = wave_sum(m) + bm[0];
        if (lane == 0) z[sg.off + i] = m;
    }
}

// ------------------------------------------------------------------ compaction
// new row dst_off + rank(i) <- old row src_off + i for tokens with keep (or all when
// keep_all): x, cat[:, :256], enc, ind.  One workgroup per (old) segment.
__global__ __launch_bounds__(256) void k_lg_compact(const int4* __restrict__ moves, const uint8_t* __restrict__ keep,
                                                    const float* __restrict__ x, const float* __restrict__ ecos,
                                                    const float* __restrict__ esin, const int32_t* __restrict__ ind,
                                                    float* __restrict__ x2, bf16_t* __restrict__ cat2,
                                                    float* __restrict__ ecos2, float* __restrict__ esin2,
                                                    int32_t* __restrict__ ind2) {
    const int4 mv = moves[blockIdx.x];  // src_off, src_len, dst_off, keep_all
    __shared__ int rank[2048 + 64];
    __shared__ int wsum[4];
    const int tid = threadIdx.x;
    // ordered ranks: 256 threads x contiguous chunks
    const int per = (mv.y + 255) / 256;
    const int a0 = tid * per, a1 = min(mv.y, a0 + per);
    int c = 0;
    for (int i = a0; i < a1; ++i) c += mv.w ? 1 : keep[mv.x + i];
    // block exclusive scan of c
    int v = c;
    const int lane = tid & 63, wave = tid >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wave; ++w) base += wsum[w];
    int r = base + v - c;
    for (int i = a0; i < a1; ++i) rank[i] = (mv.w || keep[mv.x + i]) ? r++ : -1;
    const int newlen = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    const int padded = (newlen + 63) & ~63;
    for (int e = tid; e < mv.y * LG_D; e += 256) {
        const int i = e / LG_D, cc = e % LG_D;
        const int rk = rank[i];
        if (rk < 0) continue;
        const float val = x[(size_t)(mv.x + i) * LG_D + cc];
        x2[(size_t)(mv.z + rk) * LG_D + cc] = val;
        cat2[(size_t)(mv.z + rk) * 512 + cc] = f32_to_bf16(val);
    }
    for (int e = tid; e < mv.y * 32; e += 256) {
        const int i = e / 32, f = e % 32;
        const int rk = rank[i];
        if (rk < 0) continue;
        ecos2[(size_t)(mv.z + rk) * 32 + f] = ecos[(size_t)(mv.x + i) * 32 + f];
        esin2[(size_t)(mv.z + rk) * 32 + f] = esin[(size_t)(mv.x + i) * 32 + f];
    }
    for (int i = tid; i < mv.y; i += 256)
        if (rank[i] >= 0) ind2[mv.z + rank[i]] = ind[mv.x + i];
    // zero the padding rows of the new segment
    for (int e = tid; e < (padded - newlen) * LG_D; e += 256) {
        const int i = newlen + e / LG_D, cc = e % LG_D;
        x2[(size_t)(mv.z + i) * LG_D + cc] = 0.f;
        cat2[(size_t)(mv.z + i) * 512 + cc] = 0;
    }
    for (int e = tid; e < (padded - newlen) * 32; e += 256) {
        const int i = newlen + e / 32, f = e % 32;
        ecos2[(size_t)(mv.z + i) * 32 + f] = 0.f;
        esin2[(size_t)(mv.z + i) * 32 + f] = 0.f;
    }
    for (int i = newlen + tid; i < padded; i += 256) ind2[mv.z + i] = -1;
}

__global__ void k_lg_live(const Seg* __restrict__ segs, int nseg, uint8_t* __restrict__ live, int Npad) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= Npad) return;
    uint8_t on = 0;
    for (int s = 0; s < nseg; ++s) {
        const Seg sg = segs[s];
        if (r >= sg.off && r < sg.off + sg.len) on = 1;
    }
    live[r] = on;
}

// ------------------------------------------------------------------ assignment
// S [m, n] (already / 16): row log-sum-exp, column log-sum-exp, then the row / column
// argmax of  (S - lse_row) + (S - lse_col) + (logsig(z0) + logsig(z1))  and the mutual
// filter (filter_matches).  One wave per row / column.
__global__ __launch_bounds__(256) void k_lg_row_lse(const float* __restrict__ S, int m, int n, float* __restrict__ lse) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= m) return;
    const float* row = S + (size_t)i * n;
    float mx = -INFINITY;
    for (int j = lane; j < n; j += 64) mx = fmaxf(mx, row[j]);
    mx = wave_max(mx);
    float s = 0.f;
    for (int j = lane; j < n; j += 64) s += expf(row[j] - mx);
    s = wave_sum(s);
    if (lane == 0) lse[i] = mx + logf(s);
}

__global__ __launch_bounds__(256) void k_lg_col_lse(const float* __restrict__ S, int m, int n, float* __restrict__ lse) {
    // 64 columns per workgroup; 4 waves split the rows, lanes own columns
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + lane;
    __shared__ float sm[4][64], ss[4][64];
    float mx = -INFINITY;
    if (j < n)
        for (int i = wave; i < m; i += 4) mx = fmaxf(mx, S[(size_t)i * n + j]);
    sm[wave][lane] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(sm[0][lane], sm[1][lane]), fmaxf(sm[2][lane], sm[3][lane]));
    float s = 0.f;
    if (j < n)
        for (int i = wave; i < m; i += 4) s += expf(S[(size_t)i * n + j] - mx);
    ss[wave][lane] = s;
    __syncthreads();
    if (wave == 0 && j < n) lse[j] = mx + logf(ss[0][lane] + ss[1][lane] + ss[2][lane] + ss[3][lane]);
}

__device__ __forceinline__ float lg_score(float sij, float lr, float lc, float cert) {
    return ((sij - lr) + (sij - lc)) + cert;
}

// rows: best column + value; columns: best row (first index on ties, as torch.max)
__global__ __launch_bounds__(256) void k_lg_row_arg(const float* __restrict__ S, int m, int n,
                                                    const float* __restrict__ lr, const float* __restrict__ lc,
                                                    const float* __restrict__ z0, const float* __restrict__ z1,
                                                    int* __restrict__ arg, float* __restrict__ val) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= m) return;
    const float l0 = logsigmoidf(z0[i]);
    float best = -INFINITY;
    int bj = 0x7fffffff;
    for (int j = lane; j < n; j += 64) {
        const float v = lg_score(S[(size_t)i * n + j], lr[i], lc[j], l0 + logsigmoidf(z1[j]));
        if (v > best || (v == best && j < bj)) { best = v; bj = j; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(best, o, 64);
        const int oj = __shfl_xor(bj, o, 64);
        if (ov > best || (ov == best && oj < bj)) { best = ov; bj = oj; }
    }
    if (lane == 0) { arg[i] = bj; val[i] = best; }
}

__global__ __launch_bounds__(256) void k_lg_col_arg(const float* __restrict__ S, int m, int n,
                                                    const float* __restrict__ lr, const float* __restrict__ lc,
                                                    const float* __restrict__ z0, const float* __restrict__ z1,
                                                    int* __restrict__ arg) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + lane;
    __shared__ float sb[4][64];
    __shared__ int si[4][64];
    float best = -INFINITY;
    int bi = 0x7fffffff;
    if (j < n) {
        const float l1 = logsigmoidf(z1[j]);
        for (int i = wave; i < m; i += 4) {
            const float v = lg_score(S[(size_t)i * n + j], lr[i], lc[j], logsigmoidf(z0[i]) + l1);
            if (v > best || (v == best && i < bi)) { best = v; bi = i; }
        }
    }
    sb[wave][lane] = best;
    si[wave][lane] = bi;
    __syncthreads();
    if (wave == 0 && j < n) {
        for (int w = 1; w < 4; ++w)
            if (sb[w][lane] > best || (sb[w][lane] == best && si[w][lane] < bi)) { best = sb[w][lane]; bi = si[w][lane]; }
        arg[j] = bi;
    }
}

// mutual nearest + exp(score) > th -> matches (ind0[i], ind1[m0[i]]) in row order.
// One workgroup per pair.
__global__ __launch_bounds__(256) void k_lg_filter(const int* __restrict__ a0, const float* __restrict__ v0,
                                                   const int* __restrict__ a1, int m, const int32_t* __restrict__ ind0,
                                                   const int32_t* __restrict__ ind1, float th,
                                                   int32_t* __restrict__ matches, float* __restrict__ scores,
                                                   int32_t* __restrict__ count) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ int wsum[4];
    __shared__ int base_sh;
    if (tid == 0) base_sh = 0;
    __syncthreads();
    for (int c0 = 0; c0 < m; c0 += 256) {
        const int i = c0 + tid;
        bool ok = false;
        float sc = 0.f;
        if (i < m) {
            const int j = a0[i];
            const bool mutual = a1[j] == i;
            sc = mutual ? expf(v0[i]) : 0.f;
            ok = mutual && sc > th;
        }
        int v = ok;
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(v, o, 64);
            if (lane >= o) v += t;
        }
        if (lane == 63) wsum[wave] = v;
        __syncthreads();
        int off = base_sh;
        for (int w = 0; w < wave; ++w) off += wsum[w];
        if (ok) {
            const int slot = off + v - 1;
            matches[2 * slot] = ind0[i];
            matches[2 * slot + 1] = ind1[a0[i]];
            scores[slot] = sc;
        }
        __syncthreads();
        if (tid == 0) base_sh += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
    if (tid == 0) *count = base_sh;
}

__global__ void k_scale(float* p, long n, float s) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) p[e] *= s;
}

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

struct LgLayout {
    size_t x, cat, ecos, esin, ind, x2, cat2, ecos2, esin2, ind2, qkv, Q, K, Vt, ctx, hf, hb, live, z, keep, stats,
        segs, tasks, outoff, moves, mdesc, S, lr, lc, arg0, val0, arg1, total;
};

LgLayout lg_layout(int P, int kmax) {
    const size_t N = (size_t)2 * P * (((size_t)kmax + 63) & ~(size_t)63);
    const size_t K2 = (size_t)kmax * kmax;
    LgLayout L;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += a256(bytes); return r; };
    L.x = take(N * LG_D * 4);
    L.cat = take(N * 512 * 2);
    L.ecos = take(N * 32 * 4);
    L.esin = take(N * 32 * 4);
    L.ind = take(N * 4);
    L.x2 = take(N * LG_D * 4);
    L.cat2 = take(N * 512 * 2);
    L.ecos2 = take(N * 32 * 4);
    L.esin2 = take(N * 32 * 4);
    L.ind2 = take(N * 4);
    L.qkv = take(N * 768 * 4);
    L.Q = take(N * LG_D * 2);
    L.K = take(N * LG_D * 2);
    L.Vt = take(N * LG_D * 2);
    L.ctx = take(N * LG_D * 2);
    L.hf = take(N * 512 * 4);
    L.hb = take(N * 512 * 2);
    L.live = take(N);
    L.z = take(N * 4);
    L.keep = take(N);
    L.stats = take((size_t)2 * P * 2 * 4);
    L.segs = take((size_t)2 * P * sizeof(Seg));
    L.tasks = take((size_t)4 * P * sizeof(int4));  // self tasks, then cross tasks
    L.outoff = take((size_t)4 * P * 4);
    L.moves = take((size_t)2 * P * sizeof(int4));
    L.mdesc = take(N * LG_D * 4);
    L.S = take(K2 * 4);
    L.lr = take((size_t)kmax * 4);
    L.lc = take((size_t)kmax * 4);
    L.arg0 = take((size_t)kmax * 4);
    L.val0 = take((size_t)kmax * 4);
    L.arg1 = take((size_t)kmax * 4);
    L.total = o;
    return L;
}

#define LG_TRY(x)                      \
    do {                               \
        int rc_ = (x);                 \
        if (rc_ != MLG_OK) return rc_; \
    } while (0)

float conf_threshold(int i) {
    const double t = 0.8 + 0.1 * exp(-4.0 * i / LG_L);
    return (float)std::min(1.0, std::max(0.0, t));
}

}  // namespace

size_t mlg_lightglue_ws_bytes(int P, int kmax) {
    if (P <= 0 || kmax <= 0 || kmax > 2048) return 0;
    return lg_layout(P, kmax).total;
}

int mlg_lightglue_run(const mlg_lg_weights_i& w, const float* kpts, const float* desc, const int32_t* counts, int kmax,
                      const int32_t* pa, const int32_t* pb, int P, float depth_conf, float width_conf,
                      float filter_thr, int pruning_min, void* ws, size_t ws_bytes, int32_t* matches, float* mscores,
                      int32_t* nmatch, int32_t* stop_layer, hipStream_t s) {
    if (P <= 0 || kmax <= 0 || kmax > 2048) return MLG_EINVAL;
    const LgLayout L = lg_layout(P, kmax);
    if (ws_bytes < L.total) return MLG_EINVAL;
    char* base = (char*)ws;
    float* X = (float*)(base + L.x);
    bf16_t* CAT = (bf16_t*)(base + L.cat);
    float* EC = (float*)(base + L.ecos);
    float* ES = (float*)(base + L.esin);
    int32_t* IND = (int32_t*)(base + L.ind);
    float* X2 = (float*)(base + L.x2);
    bf16_t* CAT2 = (bf16_t*)(base + L.cat2);
    float* EC2 = (float*)(base + L.ecos2);
    float* ES2 = (float*)(base + L.esin2);
    int32_t* IND2 = (int32_t*)(base + L.ind2);
    float* QKV = (float*)(base + L.qkv);
    bf16_t* Q = (bf16_t*)(base + L.Q);
    bf16_t* K = (bf16_t*)(base + L.K);
    bf16_t* VT = (bf16_t*)(base + L.Vt);
    bf16_t* CTX = (bf16_t*)(base + L.ctx);
    float* HF = (float*)(base + L.hf);
    bf16_t* HB = (bf16_t*)(base + L.hb);
    uint8_t* LIVE = (uint8_t*)(base + L.live);
    float* Z = (float*)(base + L.z);
    uint8_t* KEEP = (uint8_t*)(base + L.keep);
    int* STATS = (int*)(base + L.stats);
    Seg* SEGS = (Seg*)(base + L.segs);
    int4* TASKS = (int4*)(base + L.tasks);
    int* OUTOFF = (int*)(base + L.outoff);
    int4* MOVES = (int4*)(base + L.moves);
    float* MD = (float*)(base + L.mdesc);
    float* SS = (float*)(base + L.S);
    float* LR = (float*)(base + L.lr);
    float* LC = (float*)(base + L.lc);
    int* A0 = (int*)(base + L.arg0);
    float* V0 = (float*)(base + L.val0);
    int* A1 = (int*)(base + L.arg1);

    // Host tables below are uploaded with hipMemcpyAsync on `s` and only rewritten after
    // the stream has been synchronised (the per-layer statistics read-back), so the
    // pageable sources outlive every copy that reads them.
    std::vector<Seg> segs;
    std::vector<int> pair_of;  // pair index per active segment pair
    std::vector<int> orig_total(P);
    std::vector<int4> h_tasks;
    std::vector<int> h_out;
    std::vector<int4> h_moves;
    int off = 0;
    if (hipMemsetAsync(nmatch, 0, sizeof(int32_t) * P, s) != hipSuccess) return MLG_EHIP;
    for (int p = 0; p < P; ++p) {
        const int la = counts[pa[p]], lb = counts[pb[p]];
        if (la < 0 || la > kmax || lb < 0 || lb > kmax) return MLG_EINVAL;
        orig_total[p] = la + lb;
        if (stop_layer) stop_layer[p] = 0;
        if (la == 0 || lb == 0) continue;  // empty side: no matches (reference early exit)
        segs.push_back(Seg{off, la, pa[p], 0});
        off += (la + 63) & ~63;
        segs.push_back(Seg{off, lb, pb[p], 0});
        off += (lb + 63) & ~63;
        pair_of.push_back(p);
    }
    if (segs.empty()) return MLG_OK;
    int Npad = off;
    int maxq = 0;
    auto upload_layout = [&]() -> int {
        // segments, live-row mask, self / cross attention task lists
        h_tasks.clear();
        h_out.clear();
        maxq = 0;
        for (size_t k = 0; k < segs.size(); k += 2) {
            const Seg a = segs[k], b = segs[k + 1];
            h_tasks.push_back(make_int4(a.off, a.len, a.off, a.len));
            h_tasks.push_back(make_int4(b.off, b.len, b.off, b.len));
            maxq = std::max(maxq, std::max(a.len, b.len));
        }
        for (size_t k = 0; k < segs.size(); k += 2) {
            const Seg a = segs[k], b = segs[k + 1];
            h_tasks.push_back(make_int4(a.off, a.len, b.off, b.len));
            h_tasks.push_back(make_int4(b.off, b.len, a.off, a.len));
        }
        for (int rep = 0; rep < 2; ++rep)
            for (size_t k = 0; k < segs.size(); ++k) h_out.push_back(segs[k].off);
        if (hipMemcpyAsync(SEGS, segs.data(), segs.size() * sizeof(Seg), hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(TASKS, h_tasks.data(), h_tasks.size() * sizeof(int4), hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipMemcpyAsync(OUTOFF, h_out.data(), h_out.size() * sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess)
            return MLG_EHIP;
        hipLaunchKernelGGL(k_lg_live, dim3((Npad + 255) / 256), dim3(256), 0, s, SEGS, (int)segs.size(), LIVE, Npad);
        MLG_LAUNCH_CHECK();
        return MLG_OK;
    };
    LG_TRY(upload_layout());
    hipLaunchKernelGGL(k_lg_init, dim3((unsigned)segs.size()), dim3(256), 0, s, SEGS, kpts, desc, kmax, w.Wr, X, CAT,
                       EC, ES, IND);
    MLG_LAUNCH_CHECK();

    auto attention = [&](bool cross) -> int {
        const int nt = (int)segs.size();
        const int o = cross ? nt : 0;
        return mlg_attention_varlen(Q, cross ? Q : K, VT, CTX, LG_D, Npad, LG_H, TASKS + o, OUTOFF + o, nt, maxq, s);
    };
    auto ffn = [&](const mlg_lg_block_i& bw) -> int {
        LG_TRY(mlg_gemm_bias_bf16_ld(CTX, LG_D, bw.Wout, bw.bout, CAT + LG_D, 512, Npad, LG_D, LG_D, s));
        LG_TRY(mlg_gemm_bias_f32_ld(CAT, 512, bw.Wf1, bw.bf1, HF, 512, Npad, 512, 512, s));
        hipLaunchKernelGGL(k_lg_ln_gelu, dim3((Npad + 3) / 4), dim3(256), 0, s, HF, bw.ln_g, bw.ln_b, HB, Npad);
        LG_TRY(mlg_gemm_residual_ld(HB, 512, bw.Wf2, bw.bf2, w.ones, X, LG_D, Npad, LG_D, 512, s));
        const long n = (long)Npad * LG_D;
        hipLaunchKernelGGL(k_lg_sync, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, X, CAT, n);
        MLG_LAUNCH_CHECK();
        return MLG_OK;
    };
    // assignment + filter for the segment pair (sa, sb) of pair p at layer i
    auto assign = [&](int i, const Seg& sa, const Seg& sb, int p) -> int {
        const int m = sa.len, n = sb.len;
        float* m0 = MD + (size_t)sa.off * LG_D;
        float* m1 = MD + (size_t)sb.off * LG_D;
        LG_TRY(mlg_similarity_f32(m0, m, m1, n, LG_D, SS, n, s));
        const long nn = (long)m * n;
        hipLaunchKernelGGL(k_scale, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, s, SS, nn, 1.0f / 16.0f);
        hipLaunchKernelGGL(k_lg_row_lse, dim3((m + 3) / 4), dim3(256), 0, s, SS, m, n, LR);
        hipLaunchKernelGGL(k_lg_col_lse, dim3((n + 63) / 64), dim3(256), 0, s, SS, m, n, LC);
        hipLaunchKernelGGL(k_lg_row_arg, dim3((m + 3) / 4), dim3(256), 0, s, SS, m, n, LR, LC, Z + sa.off,
                           Z + sb.off, A0, V0);
        hipLaunchKernelGGL(k_lg_col_arg, dim3((n + 63) / 64), dim3(256), 0, s, SS, m, n, LR, LC, Z + sa.off,
                           Z + sb.off, A1);
        hipLaunchKernelGGL(k_lg_filter, dim3(1), dim3(256), 0, s, A0, V0, A1, m, IND + sa.off, IND + sb.off,
                           filter_thr, matches + (size_t)p * kmax * 2, mscores + (size_t)p * kmax, nmatch + p);
        MLG_LAUNCH_CHECK();
        if (stop_layer) stop_layer[p] = i + 1;
        (void)i;
        return MLG_OK;
    };
    auto final_proj = [&](int i) -> int {
        // mdesc = final_proj(x) for every token (the scale 1/4 per side folds into S / 16)
        return mlg_gemm_bias_f32_ld(CAT, 512, w.Wfinal[i], w.bfinal[i], MD, LG_D, Npad, LG_D, LG_D, s);
    };

    std::vector<int> stats(segs.size() * 2);
    for (int i = 0; i < LG_L && !segs.empty(); ++i) {
        // self block
        LG_TRY(mlg_gemm_bias_f32_ld(CAT, 512, w.self[i].Wqkv, w.self[i].bqkv, QKV, 768, Npad, 768, LG_D, s));
        const long nh = (long)Npad * LG_H * 32;
        hipLaunchKernelGGL(k_lg_heads_self, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, s, QKV, EC, ES, LIVE,
                           Npad, Q, K, VT);
        LG_TRY(attention(false));
        LG_TRY(ffn(w.self[i]));
        // cross block
        LG_TRY(mlg_gemm_bias_f32_ld(CAT, 512, w.cross[i].Wqkv, w.cross[i].bqkv, QKV, 512, Npad, 512, LG_D, s));
        hipLaunchKernelGGL(k_lg_heads_cross, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, s, QKV, LIVE, Npad, Q,
                           VT);
        LG_TRY(attention(true));
        LG_TRY(ffn(w.cross[i]));

        if (i == LG_L - 1) {
            LG_TRY(final_proj(i));
            hipLaunchKernelGGL(k_lg_matchability, dim3((unsigned)segs.size()), dim3(256), 0, s, SEGS, X, w.wmatch[i],
                               w.bmatch[i], Z);
            for (size_t k = 0; k < segs.size(); k += 2) LG_TRY(assign(i, segs[k], segs[k + 1], pair_of[k / 2]));
            break;
        }
        const float thr = conf_threshold(i);
        hipLaunchKernelGGL(k_lg_conf, dim3((unsigned)segs.size()), dim3(256), 0, s, SEGS, X, w.wconf[i], w.bconf[i],
                           w.wmatch[i], w.bmatch[i], thr, width_conf, Z, KEEP, STATS);
        MLG_LAUNCH_CHECK();
        if (hipMemcpyAsync(stats.data(), STATS, segs.size() * 2 * sizeof(int), hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return MLG_EHIP;
        // early stop per pair
        std::vector<char> stop(segs.size() / 2, 0);
        bool any_stop = false, any_prune = false;
        for (size_t k = 0; k < segs.size(); k += 2) {
            const int p = pair_of[k / 2];
            if (depth_conf > 0.f) {
                const float low = (float)(stats[2 * k] + stats[2 * k + 2]);
                const float ratio = 1.0f - low / (float)orig_total[p];
                if (ratio > depth_conf) {
                    stop[k / 2] = 1;
                    any_stop = true;
                }
            }
            if (!stop[k / 2] && width_conf > 0.f)
                for (int q = 0; q < 2; ++q)
                    if (segs[k + q].len > pruning_min && stats[2 * (k + q) + 1] != segs[k + q].len) any_prune = true;
        }
        if (any_stop) {
            LG_TRY(final_proj(i));
            for (size_t k = 0; k < segs.size(); k += 2)
                if (stop[k / 2]) LG_TRY(assign(i, segs[k], segs[k + 1], pair_of[k / 2]));
        }
        if (!any_stop && !any_prune) continue;
        // compact: drop stopped pairs, prune segments above the threshold
        std::vector<int4>& moves = h_moves;
        moves.clear();
        std::vector<Seg> nsegs;
        std::vector<int> npair;
        int noff = 0;
        for (size_t k = 0; k < segs.size(); k += 2) {
            if (stop[k / 2]) continue;
            for (int q = 0; q < 2; ++q) {
                const Seg sg = segs[k + q];
                const bool prune = width_conf > 0.f && sg.len > pruning_min;
                const int nl = prune ? stats[2 * (k + q) + 1] : sg.len;
                moves.push_back(make_int4(sg.off, sg.len, noff, prune ? 0 : 1));
                nsegs.push_back(Seg{noff, nl, sg.frame, 0});
                noff += (nl + 63) & ~63;
            }
            npair.push_back(pair_of[k / 2]);
        }
        if (!moves.empty()) {
            if (hipMemcpyAsync(MOVES, moves.data(), moves.size() * sizeof(int4), hipMemcpyHostToDevice, s) !=
                hipSuccess)
                return MLG_EHIP;
            hipLaunchKernelGGL(k_lg_compact, dim3((unsigned)moves.size()), dim3(256), 0, s, MOVES, KEEP, X, EC, ES,
                               IND, X2, CAT2, EC2, ES2, IND2);
            MLG_LAUNCH_CHECK();
            std::swap(X, X2);
            std::swap(CAT, CAT2);
            std::swap(EC, EC2);
            std::swap(ES, ES2);
            std::swap(IND, IND2);
        }
        // empty side after pruning -> no matches for that pair (reference loop break)
        segs.clear();
        pair_of.clear();
        for (size_t k = 0; k < nsegs.size(); k += 2) {
            if (nsegs[k].len == 0 || nsegs[k + 1].len == 0) {
                if (stop_layer) stop_layer[npair[k / 2]] = i + 2;
                continue;
            }
            segs.push_back(nsegs[k]);
            segs.push_back(nsegs[k + 1]);
            pair_of.push_back(npair[k / 2]);
        }
        Npad = std::max(noff, 64);
        if (!segs.empty()) LG_TRY(upload_layout());
        stats.assign(segs.size() * 2, 0);
    }
    return MLG_OK;
}
