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


struct Seg {
    int off, len, frame, pad;  // flat row offset, live tokens, source frame, unused
};

// ------------------------------------------------------------------ init
// normalize_keypoints without image_size: size = 1 + max - min per image,
// k' = (k - size / 2) / (max(size) / 2).  One workgroup per segment -> norm[seg] =
// (shift_x, shift_y, scale).
__global__ __launch_bounds__(256) void k_lg_kpnorm(const Seg* __restrict__ segs, const float* __restrict__ kpts,
                                                   int kmax, float4* __restrict__ norm) {
    const Seg sg = segs[blockIdx.x];
    const int tid = threadIdx.x;
    const float* kp = kpts + (size_t)sg.frame * kmax * 2;
    __shared__ float red[4][256];
    float mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
    for (int i = tid; i < sg.len; i += 256) {
        mnx = fminf(mnx, kp[2 * i]);
        mxx = fmaxf(mxx, kp[2 * i]);
        mny = fminf(mny, kp[2 * i + 1]);
        mxy = fmaxf(mxy, kp[2 * i + 1]);
    }
    red[0][tid] = mnx;
    red[1][tid] = mny;
    red[2][tid] = mxx;
    red[3][tid] = mxy;
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
    if (tid == 0) {
        const float sx = 1.f + red[2][0] - red[0][0], sy = 1.f + red[3][0] - red[1][0];
        norm[blockIdx.x] = make_float4(sx / 2.f, sy / 2.f, fmaxf(sx, sy) / 2.f, 0.f);
    }
}

// 64 rows of one segment per workgroup: Fourier positional encoding (cos / sin of
// Wr . k', 32 frequencies), x = desc, cat[:, :256] = bf16(desc), ind = source index;
// rows past len zeroed.
__global__ __launch_bounds__(256) void k_lg_init(const Seg* __restrict__ segs, const float4* __restrict__ norm,
                                                 const float* __restrict__ kpts, const float* __restrict__ desc,
                                                 int kmax, const float* __restrict__ Wr, float* __restrict__ x,
                                                 bf16_t* __restrict__ cat, float* __restrict__ ecos,
                                                 float* __restrict__ esin, int32_t* __restrict__ ind) {
    const Seg sg = segs[blockIdx.y];
    const int r0 = blockIdx.x * 64;
    if (r0 >= ((sg.len + 63) & ~63)) return;
    const float4 nm = norm[blockIdx.y];
    const float* kp = kpts + (size_t)sg.frame * kmax * 2;
    const float* ds = desc + (size_t)sg.frame * kmax * LG_D;
    for (int e = threadIdx.x; e < 64 * 32; e += 256) {
        const int i = r0 + e / 32, f = e % 32;
        const size_t r = (size_t)sg.off + i;
        const bool live = i < sg.len;
        float c = 0.f, sn = 0.f;
        if (live) {
            const float kx = (kp[2 * i] - nm.x) / nm.z, ky = (kp[2 * i + 1] - nm.y) / nm.z;
            const float pr = kx * Wr[2 * f] + ky * Wr[2 * f + 1];
            c = cosf(pr);
            sn = sinf(pr);
        }
        ecos[r * 32 + f] = c;
        esin[r * 32 + f] = sn;
        if (f == 0) ind[r] = live ? i : -1;
    }
    for (int e = threadIdx.x; e < 64 * LG_D / 4; e += 256) {
        const int i = r0 + e / (LG_D / 4), c4 = (e % (LG_D / 4)) * 4;
        const size_t r = (size_t)sg.off + i;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < sg.len) v = *reinterpret_cast<const float4*>(ds + (size_t)i * LG_D + c4);
        *reinterpret_cast<float4*>(x + r * LG_D + c4) = v;
        uint2 o;
        o.x = pack_bf16x2(v.x, v.y);
        o.y = pack_bf16x2(v.z, v.w);
        *reinterpret_cast<uint2*>(cat + r * 512 + c4) = o;
    }
}

// ------------------------------------------------------------------ confidences
// Token confidence / matchability heads run inside the cross block's fused tail
// (lg_ffn.hip, mlg_lg_conf_i): flags[r] = (conf < thr) | keep << 1, lz = logsigmoid(z).
// stats[seg] = {#(conf < thr), #keep}: one workgroup per segment
__global__ __launch_bounds__(256) void k_lg_segstats(const Seg* __restrict__ segs, const uint8_t* __restrict__ flags,
                                                     int* __restrict__ stats) {
    const Seg sg = segs[blockIdx.x];
    int low = 0, kp = 0;
    for (int i = threadIdx.x; i < sg.len; i += 256) {
        const uint8_t f = flags[sg.off + i];
        low += f & 1;
        kp += f >> 1;
    }
    low = wave_sum((float)low) + 0.5f;  // exact for counts < 2^24
    kp = wave_sum((float)kp) + 0.5f;
    __shared__ int sh[2][4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { sh[0][wave] = low; sh[1][wave] = kp; }
    __syncthreads();
    if (threadIdx.x == 0) {
        stats[2 * blockIdx.x] = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
        stats[2 * blockIdx.x + 1] = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
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
    for (int i = a0; i < a1; ++i) c += mv.w ? 1 : (keep[mv.x + i] >> 1);
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
    for (int i = a0; i < a1; ++i) rank[i] = (mv.w || (keep[mv.x + i] >> 1)) ? r++ : -1;
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

__global__ void k_lg_live(const Seg* __restrict__ segs, int nseg, uint8_t* __restrict__ live,
                          int* __restrict__ rowseg, int Npad) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= Npad) return;
    int sgi = -1;
    for (int s = 0; s < nseg; ++s) {
        const Seg sg = segs[s];
        if (r >= sg.off && r < sg.off + sg.len) sgi = s;
    }
    live[r] = sgi >= 0;
    rowseg[r] = sgi;
}

// ------------------------------------------------------------------ assignment
// For every finishing pair a (table entry Asg): S = final_proj(x0) . final_proj(x1)^T
// (f32; the two 1/4 scales applied here as one exact 1/16), the row / column
// log_softmax terms (torch form (x - max) - log(sum exp(x - max))), and the row /
// column argmax of  (s0 + s1) + (lz0 + lz1)  (first index on ties, as torch.max), then
// the mutual filter.  Row / column statistics are indexed by layout row, so all
// pairs share the buffers.  Grids carry the pair in blockIdx.y / z.
struct Asg {
    int m, n, ra, rb;  // rows of image a / b, their first layout rows
    long soff;         // S offset (floats)
    int pair, pad;
};

constexpr int CH = 256;  // rows per column-statistics chunk

// S = MD[ra .. ra + m) . MD[rb .. rb + n)^T of every listed pair in ONE launch (grid.z =
// pair; a per-pair launch left most of the chip idle on 2048 x 2048 x 256).  Exact-f32
// v_mfma_f32_32x32x2_f32 (as upstream, which runs this einsum in float32); 128 x 128
// tile, 2 x 2 waves of 64 x 64, K = 256 staged 16 at a time, transposed to [k][row].
constexpr int SBM = 128, SBK = 16;
__global__ __launch_bounds__(256, 2) void k_asg_sim(const Asg* __restrict__ tab, const float* __restrict__ MD,
                                                    float* __restrict__ Sall) {
    const Asg a = tab[blockIdx.z];
    const int m0 = blockIdx.y * SBM, n0 = blockIdx.x * SBM;
    if (m0 >= a.m || n0 >= a.n) return;
    __shared__ float As[SBK][SBM + 4];
    __shared__ float Bs[SBK][SBM + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const float* A = MD + (size_t)a.ra * LG_D;
    const float* B = MD + (size_t)a.rb * LG_D;
    f32x16 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.f;
    for (int k0 = 0; k0 < LG_D; k0 += SBK) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = tid + i * 256, row = c >> 2, kq = (c & 3) * 4;
            const float4 va = *reinterpret_cast<const float4*>(A + (size_t)min(m0 + row, a.m - 1) * LG_D + k0 + kq);
            const float4 vb = *reinterpret_cast<const float4*>(B + (size_t)min(n0 + row, a.n - 1) * LG_D + k0 + kq);
            As[kq][row] = va.x; As[kq + 1][row] = va.y; As[kq + 2][row] = va.z; As[kq + 3][row] = va.w;
            Bs[kq][row] = vb.x; Bs[kq + 1][row] = vb.y; Bs[kq + 2][row] = vb.z; Bs[kq + 3][row] = vb.w;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < SBK; kk += 2) {
            const int k = kk + (lane >> 5);
            float fa[2], fb[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                fa[t] = As[k][wm * 64 + t * 32 + (lane & 31)];
                fb[t] = Bs[k][wn * 64 + t * 32 + (lane & 31)];
            }
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[x], fb[y], acc[x][y], 0, 0, 0);
        }
        __syncthreads();
    }
    // D[i][j]: col j = lane & 31, row i = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    float* S = Sall + a.soff;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int j = n0 + wn * 64 + y * 32 + (lane & 31);
            if (j >= a.n) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = m0 + wm * 64 + x * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (i < a.m) S[(size_t)i * a.n + j] = acc[x][y][r];
            }
        }
}

__global__ __launch_bounds__(256) void k_asg_rowlse(const Asg* __restrict__ tab, const float* __restrict__ Sall,
                                                    float* __restrict__ rmax, float* __restrict__ rlog) {
    const Asg a = tab[blockIdx.y];
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.m) return;
    const float* row = Sall + a.soff + (size_t)i * a.n;
    float mx = -INFINITY;
    for (int j = lane; j < a.n; j += 64) mx = fmaxf(mx, row[j] * 0.0625f);
    mx = wave_max(mx);
    float s = 0.f;
    for (int j = lane; j < a.n; j += 64) s += expf(row[j] * 0.0625f - mx);
    s = wave_sum(s);
    if (lane == 0) {
        rmax[a.ra + i] = mx;
        rlog[a.ra + i] = logf(s);
    }
}

// per (64-column block, 256-row chunk): online (max, sum) of the column slice
__global__ __launch_bounds__(256) void k_asg_colpart(const Asg* __restrict__ tab, const float* __restrict__ Sall,
                                                     float2* __restrict__ part, int kmax) {
    const Asg a = tab[blockIdx.z];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + lane, i0 = blockIdx.y * CH;
    if ((int)blockIdx.x * 64 >= a.n || i0 >= a.m) return;
    __shared__ float2 sp[4][64];
    float mx = -INFINITY, sm = 0.f;
    if (j < a.n)
        for (int i = i0 + wave; i < min(a.m, i0 + CH); i += 4) {
            const float v = Sall[a.soff + (size_t)i * a.n + j] * 0.0625f;
            if (v > mx) {
                sm = sm * expf(mx - v) + 1.f;
                mx = v;
            } else {
                sm += expf(v - mx);
            }
        }
    sp[wave][lane] = make_float2(mx, sm);
    __syncthreads();
    if (wave == 0 && j < a.n) {
        float M = sp[0][lane].x;
        for (int w = 1; w < 4; ++w) M = fmaxf(M, sp[w][lane].x);
        float S = 0.f;
        for (int w = 0; w < 4; ++w)
            if (sp[w][lane].y > 0.f) S += sp[w][lane].y * expf(sp[w][lane].x - M);
        part[((size_t)blockIdx.z * (kmax / CH + 1) + blockIdx.y) * kmax + j] = make_float2(M, S);
    }
}

__global__ void k_asg_colfinal(const Asg* __restrict__ tab, const float2* __restrict__ part, int kmax,
                               float* __restrict__ cmax, float* __restrict__ clog) {
    const Asg a = tab[blockIdx.y];
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n) return;
    const int nch = (a.m + CH - 1) / CH;
    const float2* p = part + (size_t)blockIdx.y * (kmax / CH + 1) * kmax + j;
    float M = -INFINITY;
    for (int c = 0; c < nch; ++c) M = fmaxf(M, p[(size_t)c * kmax].x);
    float S = 0.f;
    for (int c = 0; c < nch; ++c) S += p[(size_t)c * kmax].y * expf(p[(size_t)c * kmax].x - M);
    cmax[a.rb + j] = M;
    clog[a.rb + j] = logf(S);
}

__device__ __forceinline__ float lg_score(float v, float rm, float rl, float cm, float cl, float cert) {
    return (((v - rm) - rl) + ((v - cm) - cl)) + cert;
}

__global__ __launch_bounds__(256) void k_asg_rowarg(const Asg* __restrict__ tab, const float* __restrict__ Sall,
                                                    const float* __restrict__ rmax, const float* __restrict__ rlog,
                                                    const float* __restrict__ cmax, const float* __restrict__ clog,
                                                    const float* __restrict__ lz, int* __restrict__ arg,
                                                    float* __restrict__ val) {
    const Asg a = tab[blockIdx.y];
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.m) return;
    const float* row = Sall + a.soff + (size_t)i * a.n;
    const float rm = rmax[a.ra + i], rl = rlog[a.ra + i], l0 = lz[a.ra + i];
    float best = -INFINITY;
    int bj = 0x7fffffff;
    for (int j = lane; j < a.n; j += 64) {
        const float v = lg_score(row[j] * 0.0625f, rm, rl, cmax[a.rb + j], clog[a.rb + j], l0 + lz[a.rb + j]);
        if (v > best || (v == best && j < bj)) {
            best = v;
            bj = j;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(best, o, 64);
        const int oj = __shfl_xor(bj, o, 64);
        if (ov > best || (ov == best && oj < bj)) {
            best = ov;
            bj = oj;
        }
    }
    if (lane == 0) {
        arg[a.ra + i] = bj;
        val[a.ra + i] = best;
    }
}

__global__ __launch_bounds__(256) void k_asg_colargpart(const Asg* __restrict__ tab, const float* __restrict__ Sall,
                                                        const float* __restrict__ rmax, const float* __restrict__ rlog,
                                                        const float* __restrict__ cmax, const float* __restrict__ clog,
                                                        const float* __restrict__ lz, float2* __restrict__ part,
                                                        int kmax) {
    const Asg a = tab[blockIdx.z];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + lane, i0 = blockIdx.y * CH;
    if ((int)blockIdx.x * 64 >= a.n || i0 >= a.m) return;
    __shared__ float sb[4][64];
    __shared__ int si[4][64];
    float best = -INFINITY;
    int bi = 0x7fffffff;
    if (j < a.n) {
        const float cm = cmax[a.rb + j], cl = clog[a.rb + j], l1 = lz[a.rb + j];
        for (int i = i0 + wave; i < min(a.m, i0 + CH); i += 4) {
            const float v = lg_score(Sall[a.soff + (size_t)i * a.n + j] * 0.0625f, rmax[a.ra + i], rlog[a.ra + i], cm,
                                     cl, lz[a.ra + i] + l1);
            if (v > best || (v == best && i < bi)) {
                best = v;
                bi = i;
            }
        }
    }
    sb[wave][lane] = best;
    si[wave][lane] = bi;
    __syncthreads();
    if (wave == 0 && j < a.n) {
        for (int w = 1; w < 4; ++w)
            if (sb[w][lane] > best || (sb[w][lane] == best && si[w][lane] < bi)) {
                best = sb[w][lane];
                bi = si[w][lane];
            }
        part[((size_t)blockIdx.z * (kmax / CH + 1) + blockIdx.y) * kmax + j] = make_float2(best, __int_as_float(bi));
    }
}

__global__ void k_asg_colargfinal(const Asg* __restrict__ tab, const float2* __restrict__ part, int kmax,
                                  int* __restrict__ arg) {
    const Asg a = tab[blockIdx.y];
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n) return;
    const int nch = (a.m + CH - 1) / CH;
    const float2* p = part + (size_t)blockIdx.y * (kmax / CH + 1) * kmax + j;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = 0; c < nch; ++c) {
        const float2 q = p[(size_t)c * kmax];
        const int qi = __float_as_int(q.y);
        if (q.x > best || (q.x == best && qi < bi)) {
            best = q.x;
            bi = qi;
        }
    }
    arg[a.rb + j] = bi;
}

// mutual nearest + exp(score) > th -> matches (ind0[i], ind1[m0[i]]) in row order.
// One workgroup per finishing pair.
__global__ __launch_bounds__(256) void k_lg_filter(const Asg* __restrict__ tab, const int* __restrict__ arg,
                                                   const float* __restrict__ val, const int32_t* __restrict__ ind,
                                                   float th, int kmax, int32_t* __restrict__ matches,
                                                   float* __restrict__ scores, int32_t* __restrict__ count) {
    const Asg a = tab[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ int wsum[4];
    __shared__ int base_sh;
    if (tid == 0) base_sh = 0;
    __syncthreads();
    int32_t* mo = matches + (size_t)a.pair * kmax * 2;
    float* so = scores + (size_t)a.pair * kmax;
    for (int c0 = 0; c0 < a.m; c0 += 256) {
        const int i = c0 + tid;
        bool ok = false;
        float sc = 0.f;
        int j = 0;
        if (i < a.m) {
            j = arg[a.ra + i];
            const bool mutual = arg[a.rb + j] == i;
            sc = mutual ? expf(val[a.ra + i]) : 0.f;
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
            mo[2 * slot] = ind[a.ra + i];
            mo[2 * slot + 1] = ind[a.rb + j];
            so[slot] = sc;
        }
        __syncthreads();
        if (tid == 0) base_sh += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
    if (tid == 0) count[a.pair] = base_sh;
}

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

struct LgLayout {
    size_t x, cat, ecos, esin, ind, x2, cat2, ecos2, esin2, ind2, Q, K, Vt, ctx, hf, hb, live, rowseg, lz, keep,
        stats, segs, tasks, outoff, moves, mdesc, rmax, rlog, cmax, clog, arg, val, part, asg, norm, S, total;
    int asg_cap;
};

LgLayout lg_layout(int P, int kmax) {
    const size_t N = (size_t)2 * P * (((size_t)kmax + 63) & ~(size_t)63);
    LgLayout L;
    L.asg_cap = std::min(P, 64);
    size_t o = 0;
    auto take = [&](size_t bytes) {
        size_t r = o;
        o += a256(bytes);
        return r;
    };
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
    L.Q = take(N * LG_D * 2);
    L.K = take(N * LG_D * 2);
    L.Vt = take(N * LG_D * 2);
    L.ctx = take(N * LG_D * 2);
    L.live = take(N);
    L.rowseg = take(N * 4);
    L.lz = take(N * 4);
    L.keep = take(N);
    L.stats = take((size_t)2 * P * 2 * 4);
    L.segs = take((size_t)2 * P * sizeof(Seg));
    L.tasks = take((size_t)4 * P * sizeof(int4));  // self tasks, then cross tasks
    L.outoff = take((size_t)4 * P * 4);
    L.moves = take((size_t)2 * P * sizeof(int4));
    L.mdesc = take(N * LG_D * 4);
    L.rmax = take(N * 4);
    L.rlog = take(N * 4);
    L.cmax = take(N * 4);
    L.clog = take(N * 4);
    L.arg = take(N * 4);
    L.val = take(N * 4);
    L.part = take((size_t)L.asg_cap * (kmax / CH + 1) * kmax * sizeof(float2));
    L.asg = take((size_t)P * sizeof(Asg));
    L.norm = take((size_t)2 * P * sizeof(float4));
    L.S = take((size_t)L.asg_cap * kmax * kmax * 4);
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
    bf16_t* Q = (bf16_t*)(base + L.Q);
    bf16_t* K = (bf16_t*)(base + L.K);
    bf16_t* VT = (bf16_t*)(base + L.Vt);
    bf16_t* CTX = (bf16_t*)(base + L.ctx);
    uint8_t* LIVE = (uint8_t*)(base + L.live);
    int* ROWSEG = (int*)(base + L.rowseg);
    float* LZ = (float*)(base + L.lz);
    uint8_t* KEEP = (uint8_t*)(base + L.keep);
    int* STATS = (int*)(base + L.stats);
    Seg* SEGS = (Seg*)(base + L.segs);
    int4* TASKS = (int4*)(base + L.tasks);
    int* OUTOFF = (int*)(base + L.outoff);
    int4* MOVES = (int4*)(base + L.moves);
    float* MD = (float*)(base + L.mdesc);
    float* RMAX = (float*)(base + L.rmax);
    float* RLOG = (float*)(base + L.rlog);
    float* CMAX = (float*)(base + L.cmax);
    float* CLOG = (float*)(base + L.clog);
    int* ARG = (int*)(base + L.arg);
    float* VAL = (float*)(base + L.val);
    float2* PART = (float2*)(base + L.part);
    Asg* ASG = (Asg*)(base + L.asg);
    float* SS = (float*)(base + L.S);

    // Host tables below are uploaded with hipMemcpyAsync on `s` and only rewritten after
    // the stream has been synchronised (the per-layer statistics read-back), so the
    // pageable sources outlive every copy that reads them.
    std::vector<Seg> segs;
    std::vector<int> pair_of;  // pair index per active segment pair
    std::vector<int> orig_total(P);
    std::vector<int4> h_tasks;
    std::vector<int> h_out;
    std::vector<int4> h_moves;
    std::vector<Asg> h_asg;
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
        // segments, live-row mask / row -> segment map, self and cross attention tasks
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
        hipLaunchKernelGGL(k_lg_live, dim3((Npad + 255) / 256), dim3(256), 0, s, SEGS, (int)segs.size(), LIVE, ROWSEG,
                           Npad);
        MLG_LAUNCH_CHECK();
        return MLG_OK;
    };
    LG_TRY(upload_layout());
    hipLaunchKernelGGL(k_lg_kpnorm, dim3((unsigned)segs.size()), dim3(256), 0, s, SEGS, kpts, kmax, (float4*)(base + L.norm));
    hipLaunchKernelGGL(k_lg_init, dim3((unsigned)((kmax + 63) / 64), (unsigned)segs.size()), dim3(256), 0, s, SEGS,
                       (const float4*)(base + L.norm), kpts, desc, kmax, w.Wr, X, CAT, EC, ES, IND);
    MLG_LAUNCH_CHECK();

    auto live_tokens = [&]() {
        double t = 0;
        for (const Seg& sg : segs) t += sg.len;
        return t;
    };
    auto attention = [&](bool cross) -> int {
        const int nt = (int)segs.size();
        const int o = cross ? nt : 0;
        double work = 0;  // 4 * heads * q * kv * 64 per task (QK^T and PV)
        for (size_t k = 0; k < segs.size(); k += 2) {
            const double a = segs[k].len, b = segs[k + 1].len;
            work += 4.0 * LG_H * 64 * (cross ? 2 * a * b : a * a + b * b);
        }
        MlgProfScope prof(5, s, work);
        return mlg_attention_varlen(Q, cross ? Q : K, VT, CTX, LG_D, Npad, LG_H, TASKS + o, OUTOFF + o, nt, maxq, s);
    };
    // out_proj / to_out + FFN + residual, fused (lg_ffn.hip)
    // (conf: the layer's token-confidence / matchability heads, fused into the tail)
    auto ffn = [&](const mlg_lg_block_i& bw, const mlg_lg_conf_i* conf) -> int {
        // algorithmic HBM bytes per live token: ctx + bf16 x in (512 + 512), f32 x read +
        // written (1024 + 1024), bf16 x copy written (512)
        MlgProfScope prof(8, s, 3584.0 * live_tokens());
        return mlg_lg_ffn(CTX, X, CAT, 512, Npad, bw, s, conf);
    };
    // assignment + filter of the listed segment pairs (k = index of image a's segment)
    auto assign = [&](int i, const std::vector<size_t>& ks) -> int {
        // mdesc = final_proj(x) for every token; the 1/4 per side folds into S / 16
        LG_TRY(mlg_gemm_bias_f32_ld(CAT, 512, w.Wfinal[i], w.bfinal[i], MD, LG_D, Npad, LG_D, LG_D, s));
        for (size_t c0 = 0; c0 < ks.size(); c0 += L.asg_cap) {
            const size_t c1 = std::min(ks.size(), c0 + L.asg_cap);
            if (c0 > 0 && hipStreamSynchronize(s) != hipSuccess) return MLG_EHIP;  // h_asg reuse
            h_asg.clear();
            int maxm = 0, maxn = 0;
            for (size_t c = c0; c < c1; ++c) {
                const Seg sa = segs[ks[c]], sb = segs[ks[c] + 1];
                Asg a;
                a.m = sa.len;
                a.n = sb.len;
                a.ra = sa.off;
                a.rb = sb.off;
                a.soff = (long)(c - c0) * kmax * kmax;
                a.pair = pair_of[ks[c] / 2];
                a.pad = 0;
                h_asg.push_back(a);
                maxm = std::max(maxm, a.m);
                maxn = std::max(maxn, a.n);
                if (stop_layer) stop_layer[a.pair] = i + 1;
            }
            const unsigned na = (unsigned)h_asg.size();
            if (hipMemcpyAsync(ASG, h_asg.data(), na * sizeof(Asg), hipMemcpyHostToDevice, s) != hipSuccess)
                return MLG_EHIP;
            hipLaunchKernelGGL(k_asg_sim, dim3((maxn + SBM - 1) / SBM, (maxm + SBM - 1) / SBM, na), dim3(256), 0, s, ASG,
                               MD, SS);
            const dim3 rows((maxm + 3) / 4, na), cols((maxn + 63) / 64, (maxm + CH - 1) / CH, na),
                cfin((maxn + 255) / 256, na);
            hipLaunchKernelGGL(k_asg_rowlse, rows, dim3(256), 0, s, ASG, SS, RMAX, RLOG);
            hipLaunchKernelGGL(k_asg_colpart, cols, dim3(256), 0, s, ASG, SS, PART, kmax);
            hipLaunchKernelGGL(k_asg_colfinal, cfin, dim3(256), 0, s, ASG, PART, kmax, CMAX, CLOG);
            hipLaunchKernelGGL(k_asg_rowarg, rows, dim3(256), 0, s, ASG, SS, RMAX, RLOG, CMAX, CLOG, LZ, ARG, VAL);
            hipLaunchKernelGGL(k_asg_colargpart, cols, dim3(256), 0, s, ASG, SS, RMAX, RLOG, CMAX, CLOG, LZ, PART,
                               kmax);
            hipLaunchKernelGGL(k_asg_colargfinal, cfin, dim3(256), 0, s, ASG, PART, kmax, ARG);
            hipLaunchKernelGGL(k_lg_filter, dim3(na), dim3(256), 0, s, ASG, ARG, VAL, IND, filter_thr, kmax, matches,
                               mscores, nmatch);
            MLG_LAUNCH_CHECK();
        }
        return MLG_OK;
    };

    std::vector<int> stats(segs.size() * 2);
    for (int i = 0; i < LG_L && !segs.empty(); ++i) {
        // self block: projection + rotary + head split fused in the GEMM epilogue
        {
            MlgProfScope prof(6, s, 2.0 * live_tokens() * 768 * 256);
            LG_TRY(mlg_lg_proj(true, CAT, 512, w.self[i].Wqkv, w.self[i].bqkv, EC, ES, LIVE, Q, K, VT, Npad, s));
        }
        LG_TRY(attention(false));
        LG_TRY(ffn(w.self[i], nullptr));
        // cross block
        {
            MlgProfScope prof(6, s, 2.0 * live_tokens() * 512 * 256);
            LG_TRY(mlg_lg_proj(false, CAT, 512, w.cross[i].Wqkv, w.cross[i].bqkv, nullptr, nullptr, LIVE, Q, nullptr, VT,
                               Npad, s));
        }
        LG_TRY(attention(true));
        // layer i's heads on the updated tokens: matchability log-sigmoid (the assignment's
        // certainty term) and, before the last layer, confidences + early-stop / prune flags
        const bool last = i == LG_L - 1;
        const mlg_lg_conf_i heads{ROWSEG, last ? nullptr : w.wconf[i], last ? nullptr : w.bconf[i], w.wmatch[i],
                                  w.bmatch[i], last ? 0.f : conf_threshold(i), width_conf, LZ, KEEP};
        LG_TRY(ffn(w.cross[i], &heads));

        if (last) {
            std::vector<size_t> ks;
            for (size_t k = 0; k < segs.size(); k += 2) ks.push_back(k);
            LG_TRY(assign(i, ks));
            break;
        }
        hipLaunchKernelGGL(k_lg_segstats, dim3((unsigned)segs.size()), dim3(256), 0, s, SEGS, KEEP, STATS);
        MLG_LAUNCH_CHECK();
        if (hipMemcpyAsync(stats.data(), STATS, segs.size() * 2 * sizeof(int), hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return MLG_EHIP;
        // early stop per pair; point pruning per segment
        std::vector<char> stop(segs.size() / 2, 0);
        std::vector<size_t> stopped;
        bool any_prune = false;
        for (size_t k = 0; k < segs.size(); k += 2) {
            const int p = pair_of[k / 2];
            if (depth_conf > 0.f) {
                const float low = (float)(stats[2 * k] + stats[2 * k + 2]);
                const float ratio = 1.0f - low / (float)orig_total[p];
                if (ratio > depth_conf) {
                    stop[k / 2] = 1;
                    stopped.push_back(k);
                }
            }
            if (!stop[k / 2] && width_conf > 0.f)
                for (int q = 0; q < 2; ++q)
                    if (segs[k + q].len > pruning_min && stats[2 * (k + q) + 1] != segs[k + q].len) any_prune = true;
        }
        if (!stopped.empty()) LG_TRY(assign(i, stopped));  // the matchability lz came with the confidences
        if (stopped.empty() && !any_prune) continue;
        // compact: drop stopped pairs, prune segments above the threshold
        h_moves.clear();
        std::vector<Seg> nsegs;
        std::vector<int> npair;
        int noff = 0;
        for (size_t k = 0; k < segs.size(); k += 2) {
            if (stop[k / 2]) continue;
            for (int q = 0; q < 2; ++q) {
                const Seg sg = segs[k + q];
                const bool prune = width_conf > 0.f && sg.len > pruning_min;
                const int nl = prune ? stats[2 * (k + q) + 1] : sg.len;
                h_moves.push_back(make_int4(sg.off, sg.len, noff, prune ? 0 : 1));
                nsegs.push_back(Seg{noff, nl, sg.frame, 0});
                noff += (nl + 63) & ~63;
            }
            npair.push_back(pair_of[k / 2]);
        }
        if (!h_moves.empty()) {
            if (!stopped.empty() && hipStreamSynchronize(s) != hipSuccess) return MLG_EHIP;  // h_asg in flight
            if (hipMemcpyAsync(MOVES, h_moves.data(), h_moves.size() * sizeof(int4), hipMemcpyHostToDevice, s) !=
                hipSuccess)
                return MLG_EHIP;
            hipLaunchKernelGGL(k_lg_compact, dim3((unsigned)h_moves.size()), dim3(256), 0, s, MOVES, KEEP, X, EC, ES,
                               IND, X2, CAT2, EC2, ES2, IND2);
            MLG_LAUNCH_CHECK();
            std::swap(X, X2);
            std::swap(CAT, CAT2);
            std::swap(EC, EC2);
            std::swap(ES, ES2);
            std::swap(IND, IND2);
        }
        // an empty side after pruning ends that pair with no matches (reference loop break)
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
