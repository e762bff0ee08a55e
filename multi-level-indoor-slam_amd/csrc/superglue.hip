// SuperGlue matcher with log-space optimal transport (Sinkhorn): the configuration of the
// reference's SuperGlue class (scripts/semantic_gating/geometric_verification.py:353-421:
// SuperPoint nms_radius 4 / keypoint_threshold 0.005, SuperGlue weights 'indoor',
// sinkhorn_iterations 20, match_threshold 0.2), whose native branch the reference never
// reaches (:419-421 defer to a fallback); semantics of magicleap's models/superglue.py
// restated in oracle/superglue.py.
//
// Over a ragged batch of pairs in LightGlue's flat token layout (segments padded to 64
// rows), reusing its kernels:
//   k_sg_gather    descriptors -> f32 residual stream rows, normalised keypoints
//                  ((k - size / 2) / (0.7 max(W, H))) + score -> the keypoint encoder's
//                  first three layers (3 -> 32 -> 64 -> 128, BatchNorm folded, ReLU) on
//                  the VALU, bf16;
//   mlg_gemm_conv  encoder layers 4 (128 -> 256, BN + ReLU) and 5 (256 -> 256, + the
//                  descriptor as residual): x = desc + kenc, f32 and its bf16 copy;
//   18 GNN layers  (self / cross alternating): mlg_lg_proj (q, k, v with biases, heads
//                  made contiguous by a row permutation on the host; identity rotary),
//                  k_attention_varlen (self: seg -> seg; cross: a -> b, b -> a; both from
//                  the pre-layer states, as AttentionalGNN), mlg_lg_ffn in ReLU mode
//                  (merge + MLP [x | msg] 512 -> 512 (BN folded) -> ReLU -> 256 + residual);
//   final_proj     GEMM -> f32 matching descriptors;
//   per pair       S = m0 . m1^T and T = S^T on the exact-f32 MFMA (one kernel, chunks
//                  of pairs); Z =
//                  S / 16 with the learned dustbin score on the extra row / column; 20
//                  log-Sinkhorn iterations (k_sg_lse<false>: u = log_mu - logsumexp_j(Z + v)
//                  over rows of S; k_sg_lse<true>: v = log_nu - logsumexp_i(Z + u) over rows
//                  of T); k_sg_argmax<false / true> on Z + u + v - norm; k_sg_select:
//                  mutual nearest, exp(score) > threshold, compacted.
#include <math.h>

#include <algorithm>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace {

struct SgSeg {
    int off, len, frame, pad;
};

// k_sg_gather: row r of segment s (token t of frame f) -> X[r] = desc[f][t] (f32),
// h3[r] = kenc layers 1-3 on (x, y, score) (bf16, 128).  Dead rows: zeros.
__global__ __launch_bounds__(128) void k_sg_gather(const SgSeg* __restrict__ segs, int nseg, int Npad,
                                                   const float* __restrict__ kpts, const float* __restrict__ kscores,
                                                   const float* __restrict__ desc, int kmax, float W, float H,
                                                   const float* __restrict__ w1, const float* __restrict__ b1,
                                                   const float* __restrict__ w2, const float* __restrict__ b2,
                                                   const float* __restrict__ w3, const float* __restrict__ b3,
                                                   float* __restrict__ X, bf16_t* __restrict__ h3) {
    __shared__ float s_in[3], s_h1[32], s_h2[64];
    const int r = blockIdx.x, tid = threadIdx.x;
    // segment lookup (segments in increasing offset order)
    int lo = 0, hi = nseg - 1, sg = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (segs[mid].off <= r) {
            sg = mid;
            lo = mid + 1;
        } else {
            hi = mid - 1;
        }
    }
    const bool live = sg >= 0 && r < segs[sg].off + segs[sg].len;
    float* xr = X + (size_t)r * 256;
    bf16_t* hr = h3 + (size_t)r * 128;
    if (!live) {
        xr[tid] = 0.f;
        xr[tid + 128] = 0.f;
        hr[tid] = 0;
        return;
    }
    const int f = segs[sg].frame, t = r - segs[sg].off;
    const float* d = desc + ((size_t)f * kmax + t) * 256;
    xr[tid] = d[tid];
    xr[tid + 128] = d[tid + 128];
    if (tid == 0) {
        const float* k = kpts + ((size_t)f * kmax + t) * 2;
        const float sc = fmaxf(W, H) * 0.7f;
        s_in[0] = (k[0] - W / 2.f) / sc;
        s_in[1] = (k[1] - H / 2.f) / sc;
        s_in[2] = kscores[(size_t)f * kmax + t];
    }
    __syncthreads();
    if (tid < 32) {
        float a = b1[tid];
        for (int i = 0; i < 3; ++i) a = fmaf(w1[tid * 3 + i], s_in[i], a);
        s_h1[tid] = fmaxf(a, 0.f);
    }
    __syncthreads();
    if (tid < 64) {
        float a = b2[tid];
        for (int i = 0; i < 32; ++i) a = fmaf(w2[tid * 32 + i], s_h1[i], a);
        s_h2[tid] = fmaxf(a, 0.f);
    }
    __syncthreads();
    float a = b3[tid];
    for (int i = 0; i < 64; ++i) a = fmaf(w3[tid * 64 + i], s_h2[i], a);
    hr[tid] = f32_to_bf16(fmaxf(a, 0.f));
}

// the identity rotation (cos 1, sin 0) in the projections' lg_fac4 factor layout: every
// float4 = (cos, cos, sin, sin) = (1, 1, 0, 0) -- the self-block projection with no rotary
__global__ void k_sg_fill_rot(float4* __restrict__ a, long n) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) a[e] = make_float4(1.f, 1.f, 0.f, 0.f);
}

// ------------------------------------------------------------- Sinkhorn -----
// Pair c of a chunk: S_c [m][n] and its transpose T_c [n][m] (row stride ld each) ->
// Z_ij = S_ij / 16 (i < m, j < n), the dustbin row / column and corner = alpha.  u [m + 1]
// and v [n + 1] of every pair live in two flat vectors (offsets uo, vo).  With the
// transpose stored, the u update (logsumexp over a row of Z + v) and the v update (over a
// column of Z + u) are the same row-wise pass: coalesced 16-B loads, one wave per row.
struct SgPair {
    int m, n, uo, vo, pid, pad0, pad1, pad2;
};

__device__ __forceinline__ void lse_merge(float omx, float osm, float& mx, float& sm) {
    if (omx > mx) {
        sm = sm * expf(mx - omx) + osm;
        mx = omx;
    } else if (omx > -INFINITY) {
        sm += osm * expf(omx - mx);
    }
}

// TR = false: u_i = log_mu_i - logsumexp_j (Z_ij + v_j), rows i in [0, m] of S;
// TR = true : v_j = log_nu_j - logsumexp_i (Z_ij + u_i), rows j in [0, n] of T.
template <bool TR>
__global__ __launch_bounds__(256) void k_sg_lse(const float* __restrict__ S, long sstride, int ld,
                                                const SgPair* __restrict__ pairs, float alpha, float* __restrict__ out,
                                                const float* __restrict__ in) {
    const int c = blockIdx.y, lane = threadIdx.x & 63;
    const SgPair p = pairs[c];
    const int R = TR ? p.n : p.m, C = TR ? p.m : p.n;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i > R) return;
    const float* inv = in + (TR ? p.uo : p.vo);
    float mx = -INFINITY, sm = 0.f;
    if (i < R) {
        // blocks of 2048 columns held in registers (8 float4 per lane): block max, one
        // rescale, one exp per element
        const float* row = S + (size_t)c * sstride + (size_t)i * ld;
        for (int base = 0; base < C; base += 2048) {
            float x[8][4];
            float bm = -INFINITY;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int j0 = base + 256 * t + 4 * lane;
                float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f), v4 = s4;
                if (j0 < C) {
                    s4 = *reinterpret_cast<const float4*>(row + j0);
                    v4 = *reinterpret_cast<const float4*>(inv + j0);
                }
                x[t][0] = j0 < C ? s4.x * 0.0625f + v4.x : -INFINITY;
                x[t][1] = j0 + 1 < C ? s4.y * 0.0625f + v4.y : -INFINITY;
                x[t][2] = j0 + 2 < C ? s4.z * 0.0625f + v4.z : -INFINITY;
                x[t][3] = j0 + 3 < C ? s4.w * 0.0625f + v4.w : -INFINITY;
                bm = fmaxf(bm, fmaxf(fmaxf(x[t][0], x[t][1]), fmaxf(x[t][2], x[t][3])));
            }
            if (bm > mx) {
                sm *= expf(mx - bm);
                mx = bm;
            }
            if (mx > -INFINITY) {
#pragma unroll
                for (int t = 0; t < 8; ++t)
#pragma unroll
                    for (int k = 0; k < 4; ++k) sm += expf(x[t][k] - mx);
            }
        }
        if (lane == 0) lse_merge(alpha + inv[C], 1.f, mx, sm);  // dustbin column
    } else {  // dustbin row: alpha everywhere
        for (int j = lane; j <= C; j += 64) lse_merge(alpha + inv[j], 1.f, mx, sm);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float omx = __shfl_xor(mx, o, 64), osm = __shfl_xor(sm, o, 64);
        lse_merge(omx, osm, mx, sm);
    }
    if (lane == 0) {
        const float norm = -logf((float)(p.m + p.n));
        const float lm = i < R ? norm : logf((float)C) + norm;
        out[(TR ? p.vo : p.uo) + i] = lm - (mx + logf(sm));
    }
}

// argmax over the inner block of Z + u + v - norm (first index on ties), one wave per
// row: TR = false rows i of S (-> value and column index), TR = true rows j of T (-> row
// index).  Both evaluate ((S_ij / 16 + u_i) + v_j) - norm, as torch does.
template <bool TR>
__global__ __launch_bounds__(256) void k_sg_argmax(const float* __restrict__ S, long sstride, int ld,
                                                   const SgPair* __restrict__ pairs, const float* __restrict__ u,
                                                   const float* __restrict__ v, float* __restrict__ vmax,
                                                   int32_t* __restrict__ idx, int kmax) {
    const int c = blockIdx.y, lane = threadIdx.x & 63;
    const SgPair p = pairs[c];
    const int R = TR ? p.n : p.m, C = TR ? p.m : p.n;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= R) return;
    const float* row = S + (size_t)c * sstride + (size_t)i * ld;
    const float* uc = u + p.uo;
    const float* vc = v + p.vo;
    const float norm = -logf((float)(p.m + p.n));
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int j = lane; j < C; j += 64) {
        const float z = TR ? ((row[j] * 0.0625f + uc[j]) + vc[i]) - norm : ((row[j] * 0.0625f + uc[i]) + vc[j]) - norm;
        if (z > bv) {
            bv = z;
            bi = j;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) {
            bv = ov;
            bi = oi;
        }
    }
    if (lane == 0) {
        if (!TR) vmax[(size_t)c * kmax + i] = bv;
        idx[(size_t)c * kmax + i] = bi;
    }
}

// mutual nearest + exp(score) > thr, compacted in row order; one workgroup per pair
__global__ __launch_bounds__(1024) void k_sg_select(const SgPair* __restrict__ pairs, const float* __restrict__ rmax,
                                                    const int32_t* __restrict__ ridx,
                                                    const int32_t* __restrict__ cidx, int kmax, float thr,
                                                    int32_t* __restrict__ matches,
                                                    float* __restrict__ mscores, int32_t* __restrict__ nmatch) {
    __shared__ int warp_tot[16];
    __shared__ int base;
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const SgPair p = pairs[c];
    const int pid = p.pid;
    if (tid == 0) base = 0;
    __syncthreads();
    for (int i0 = 0; i0 < p.m; i0 += 1024) {
        const int i = i0 + tid;
        bool ok = false;
        int j = 0;
        float sc = 0.f;
        if (i < p.m) {
            j = ridx[(size_t)c * kmax + i];
            if (j >= 0 && j < p.n && cidx[(size_t)c * kmax + j] == i) {
                sc = expf(rmax[(size_t)c * kmax + i]);
                ok = sc > thr;
            }
        }
        const unsigned long long bal = __ballot(ok);
        const int pre = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) warp_tot[wave] = __popcll(bal);
        __syncthreads();
        int off = base;
        for (int w = 0; w < wave; ++w) off += warp_tot[w];
        if (ok) {
            const size_t o = (size_t)pid * kmax + off + pre;
            matches[2 * o] = i;
            matches[2 * o + 1] = j;
            mscores[o] = sc;
        }
        __syncthreads();
        if (tid == 0) {
            int t = 0;
            for (int w = 0; w < 16; ++w) t += warp_tot[w];
            base += t;
        }
        __syncthreads();
    }
    if (tid == 0) nmatch[pid] = base;
}

inline size_t a256(size_t b) { return (b + 255) & ~(size_t)255; }

// pairs per Sinkhorn chunk: S and T of a chunk within SG_CHUNK_MB (larger launches
// amortise the ramp; 128 MB would keep them in the 256 MB last-level cache), at most 64
#ifndef SG_CHUNK_MB
#define SG_CHUNK_MB 512
#endif
inline int sg_chunk(int kmax) {
    const size_t per = (size_t)2 * kmax * (((size_t)kmax + 3) & ~(size_t)3) * 4;
    return (int)std::max<size_t>(1, std::min<size_t>(64, ((size_t)SG_CHUNK_MB << 20) / per));
}

struct SgLayout {
    size_t x, cat, Q, K, Vt, ctx, h3, h4, live, ef, md, segs, tasks, outoff, S, T, u, v, pairs, rmax, ridx, cidx,
        total;
};

SgLayout sg_layout(int P, int kmax) {
    const size_t N = (size_t)2 * P * (((size_t)kmax + 63) & ~(size_t)63);
    const size_t ldS = ((size_t)kmax + 3) & ~(size_t)3;
    const size_t ch = (size_t)sg_chunk(kmax);
    SgLayout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) {
        size_t r = o;
        o += a256(bytes);
        return r;
    };
    L.x = take(N * 256 * 4);
    L.cat = take(N * 512 * 2);
    L.Q = take(N * 256 * 2);
    L.K = take(N * 256 * 2);
    L.Vt = take(N * 256 * 2);
    L.ctx = take(N * 256 * 2);
    L.h3 = take(N * 128 * 2);
    L.h4 = take(N * 256 * 2);
    L.live = take(N);
    L.ef = take(N * 64 * 4);
    L.md = take(N * 256 * 4);
    L.segs = take((size_t)2 * P * sizeof(SgSeg));
    L.tasks = take((size_t)4 * P * sizeof(int4));
    L.outoff = take((size_t)4 * P * 4);
    L.S = take(ch * kmax * ldS * 4);
    L.T = take(ch * kmax * ldS * 4);
    L.u = take((size_t)P * (kmax + 4) * 4);
    L.v = take((size_t)P * (kmax + 4) * 4);
    L.pairs = take((size_t)P * sizeof(SgPair));
    L.rmax = take(ch * kmax * 4);
    L.ridx = take(ch * kmax * 4);
    L.cidx = take(ch * kmax * 4);
    L.total = o;
    return L;
}

__global__ void k_sg_live(const SgSeg* __restrict__ segs, int nseg, uint8_t* __restrict__ live, int Npad) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= Npad) return;
    int lo = 0, hi = nseg - 1, sg = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (segs[mid].off <= r) {
            sg = mid;
            lo = mid + 1;
        } else {
            hi = mid - 1;
        }
    }
    live[r] = sg >= 0 && r < segs[sg].off + segs[sg].len;
}

#define SG_TRY(x)                      \
    do {                               \
        int rc_ = (x);                 \
        if (rc_ != MLG_OK) return rc_; \
    } while (0)

}  // namespace

size_t mlg_superglue_ws_bytes(int P, int kmax) {
    if (P <= 0 || kmax <= 0) return 0;
    return sg_layout(P, kmax).total;
}

int mlg_superglue_run(const mlg_sg_weights_i& w, const float* kpts, const float* kscores, const float* desc,
                      const int32_t* counts, int kmax, int W, int H, const int32_t* pa, const int32_t* pb, int P,
                      int iters, float thr, void* ws, size_t ws_bytes, int32_t* matches, float* mscores,
                      int32_t* nmatch, hipStream_t s) {
    if (P <= 0 || kmax <= 0 || !kpts || !kscores || !desc || !counts || !pa || !pb || !matches || !mscores ||
        !nmatch || iters < 0)
        return MLG_EINVAL;
    const SgLayout L = sg_layout(P, kmax);
    if (ws_bytes < L.total) return MLG_EINVAL;
    char* base = (char*)ws;
    auto at = [&](size_t off) { return (void*)(base + off); };
    float* X = (float*)at(L.x);
    bf16_t* CAT = (bf16_t*)at(L.cat);
    bf16_t* Q = (bf16_t*)at(L.Q);
    bf16_t* K = (bf16_t*)at(L.K);
    bf16_t* VT = (bf16_t*)at(L.Vt);
    bf16_t* CTX = (bf16_t*)at(L.ctx);
    bf16_t* H3 = (bf16_t*)at(L.h3);
    bf16_t* H4 = (bf16_t*)at(L.h4);
    uint8_t* LIVE = (uint8_t*)at(L.live);
    float* EF = (float*)at(L.ef);  // identity rotary factors (lg_fac4 layout)
    float* MD = (float*)at(L.md);
    SgSeg* SEGS = (SgSeg*)at(L.segs);
    int4* TASKS = (int4*)at(L.tasks);
    int* OUTOFF = (int*)at(L.outoff);
    float* S = (float*)at(L.S);
    float* T = (float*)at(L.T);
    float* U = (float*)at(L.u);
    float* V = (float*)at(L.v);
    SgPair* PAIRS = (SgPair*)at(L.pairs);
    float* RMAX = (float*)at(L.rmax);
    int32_t* RIDX = (int32_t*)at(L.ridx);
    int32_t* CIDX = (int32_t*)at(L.cidx);

    if (hipMemsetAsync(nmatch, 0, sizeof(int32_t) * P, s) != hipSuccess) return MLG_EHIP;
    // segments: pair p -> [a | b], empty sides skipped (no matches, as the reference's early exit)
    std::vector<SgSeg> segs;
    std::vector<int> pair_of;
    int off = 0;
    for (int p = 0; p < P; ++p) {
        const int la = counts[pa[p]], lb = counts[pb[p]];
        if (la < 0 || la > kmax || lb < 0 || lb > kmax) return MLG_EINVAL;
        if (la == 0 || lb == 0) continue;
        segs.push_back(SgSeg{off, la, pa[p], 0});
        off += (la + 63) & ~63;
        segs.push_back(SgSeg{off, lb, pb[p], 0});
        off += (lb + 63) & ~63;
        pair_of.push_back(p);
    }
    if (segs.empty()) return hipStreamSynchronize(s) == hipSuccess ? MLG_OK : MLG_EHIP;
    const int Npad = off, nseg = (int)segs.size(), np = nseg / 2;
    std::vector<int4> h_tasks;
    std::vector<int> h_out;
    int maxq = 0;
    for (int k = 0; k < nseg; ++k) {
        h_tasks.push_back(make_int4(segs[k].off, segs[k].len, segs[k].off, segs[k].len));
        maxq = std::max(maxq, segs[k].len);
    }
    for (int k = 0; k < nseg; k += 2) {
        h_tasks.push_back(make_int4(segs[k].off, segs[k].len, segs[k + 1].off, segs[k + 1].len));
        h_tasks.push_back(make_int4(segs[k + 1].off, segs[k + 1].len, segs[k].off, segs[k].len));
    }
    for (int rep = 0; rep < 2; ++rep)
        for (int k = 0; k < nseg; ++k) h_out.push_back(segs[k].off);
    if (hipMemcpyAsync(SEGS, segs.data(), segs.size() * sizeof(SgSeg), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(TASKS, h_tasks.data(), h_tasks.size() * sizeof(int4), hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipMemcpyAsync(OUTOFF, h_out.data(), h_out.size() * sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess)
        return MLG_EHIP;
    hipLaunchKernelGGL(k_sg_live, dim3((Npad + 255) / 256), dim3(256), 0, s, SEGS, nseg, LIVE, Npad);
    hipLaunchKernelGGL(k_sg_fill_rot, dim3((unsigned)(((long)Npad * 16 + 255) / 256)), dim3(256), 0, s,
                       (float4*)EF, (long)Npad * 16);
    // keypoint encoder: layers 1-3 on the VALU, 4-5 as GEMMs; x = desc + kenc
    hipLaunchKernelGGL(k_sg_gather, dim3(Npad), dim3(128), 0, s, SEGS, nseg, Npad, kpts, kscores, desc, kmax,
                       (float)W, (float)H, w.kenc_w[0], w.kenc_b[0], w.kenc_w[1], w.kenc_b[1], w.kenc_w[2],
                       w.kenc_b[2], X, H3);
    MLG_LAUNCH_CHECK();
    SG_TRY(mlg_gemm_conv(H3, 128, w.kenc_w4, w.kenc_b4, nullptr, 0, nullptr, 0, H4, 256, 1, 256, Npad, 256, 128, s));
    SG_TRY(mlg_gemm_conv(H4, 256, w.kenc_w5, w.kenc_b5, X, 256, X, 256, CAT, 512, 0, 0, Npad, 256, 256, s));
    // the GNN: 18 layers, self / cross alternating, every projection from the pre-layer states
    for (int l = 0; l < 18; ++l) {
        const bool cross = (l & 1) != 0;
        SG_TRY(mlg_lg_proj(true, CAT, 512, w.layer[l].Wqkv, w.layer[l].bqkv, EF, LIVE, Q, K, VT, Npad, s));
        SG_TRY(mlg_attention_varlen(Q, K, VT, CTX, 256, Npad, 4, TASKS + (cross ? nseg : 0),
                                    OUTOFF + (cross ? nseg : 0), nseg, maxq, s));
        SG_TRY(mlg_lg_ffn(CTX, X, CAT, 512, Npad, w.layer[l], s, nullptr, 1));
    }
    // matching descriptors
    SG_TRY(mlg_gemm_conv(CAT, 512, w.Wfinal, w.bfinal, nullptr, 0, MD, 256, nullptr, 0, 0, 0, Npad, 256, 256, s));
    // per chunk of pairs: scores and their transpose, Sinkhorn, mutual matches
    const int ldS = (kmax + 3) & ~3;
    const long sstride = (long)kmax * ldS;
    const int chunk = sg_chunk(kmax);
    std::vector<SgPair> hp(np);
    int uo = 0, vo = 0;
    for (int c = 0; c < np; ++c) {
        const SgSeg a = segs[2 * c], b = segs[2 * c + 1];
        hp[c] = SgPair{a.len, b.len, uo, vo, pair_of[c], 0, 0, 0};
        uo += (a.len + 4) & ~3;  // 16-B aligned vectors
        vo += (b.len + 4) & ~3;
    }
    if (hipMemcpyAsync(PAIRS, hp.data(), np * sizeof(SgPair), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(U, 0, (size_t)uo * 4, s) != hipSuccess || hipMemsetAsync(V, 0, (size_t)vo * 4, s) != hipSuccess)
        return MLG_EHIP;
    for (int c0 = 0; c0 < np; c0 += chunk) {
        const int nc = std::min(chunk, np - c0);
        int mm = 0, nn = 0;
        for (int c = 0; c < nc; ++c) {
            const SgSeg a = segs[2 * (c0 + c)], b = segs[2 * (c0 + c) + 1];
            mm = std::max(mm, a.len);
            nn = std::max(nn, b.len);
            SG_TRY(mlg_similarity_f32_t(MD + (size_t)a.off * 256, a.len, MD + (size_t)b.off * 256, b.len, 256,
                                        S + (size_t)c * sstride, ldS, T + (size_t)c * sstride, ldS, s));
        }
        const SgPair* pc = PAIRS + c0;
        const dim3 rows((mm + 1 + 3) / 4, nc), cols((nn + 1 + 3) / 4, nc);
        for (int it = 0; it < iters; ++it) {
            hipLaunchKernelGGL(k_sg_lse<false>, rows, dim3(256), 0, s, S, sstride, ldS, pc, w.bin_score, U, V);
            hipLaunchKernelGGL(k_sg_lse<true>, cols, dim3(256), 0, s, T, sstride, ldS, pc, w.bin_score, V, U);
        }
        hipLaunchKernelGGL(k_sg_argmax<false>, dim3((mm + 3) / 4, nc), dim3(256), 0, s, S, sstride, ldS, pc, U, V,
                           RMAX, RIDX, kmax);
        hipLaunchKernelGGL(k_sg_argmax<true>, dim3((nn + 3) / 4, nc), dim3(256), 0, s, T, sstride, ldS, pc, U, V,
                           (float*)nullptr, CIDX, kmax);
        hipLaunchKernelGGL(k_sg_select, dim3(nc), dim3(1024), 0, s, pc, RMAX, RIDX, CIDX, kmax, thr, matches, mscores,
                           nmatch);
        MLG_LAUNCH_CHECK();
    }
    // the segment / task / pair tables are pageable host vectors
    return hipStreamSynchronize(s) == hipSuccess ? MLG_OK : MLG_EHIP;
}
