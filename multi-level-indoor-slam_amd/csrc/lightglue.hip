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
#include <unordered_map>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "../../include/mlgate.h"

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

#ifndef MLG_LG_INIT_FUSED
#define MLG_LG_INIT_FUSED 1  // 0: the separate k_lg_gather_rows pass (A/B only)
#endif

// 64 rows of one segment per workgroup: Fourier positional encoding (cos / sin of
// Wr . k', 32 frequencies), x = desc, cat[:, :256] = bf16(desc), ind = source index;
// rows past len zeroed.  With mv (layer 0's self block already run per frame): the live
// rows' x and bf16 copy come from that block's output instead, mv[seg] = (pair offset,
// live rows, frame offset, -) -- k_lg_gather_rows folded into this pass.
__global__ __launch_bounds__(256) void k_lg_init(const Seg* __restrict__ segs, const float4* __restrict__ norm,
                                                 const float* __restrict__ kpts, const float* __restrict__ desc,
                                                 int kmax, const float* __restrict__ Wr, float* __restrict__ x,
                                                 bf16_t* __restrict__ cat, float4* __restrict__ efac,
                                                 int32_t* __restrict__ ind,
                                                 const int4* __restrict__ mv = nullptr,
                                                 const float* __restrict__ xf = nullptr,
                                                 const bf16_t* __restrict__ catf = nullptr) {
    const Seg sg = segs[blockIdx.y];
    const int r0 = blockIdx.x * 64;
    if (r0 >= ((sg.len + 63) & ~63)) return;
    const float4 nm = norm[blockIdx.y];
    const float* kp = kpts + (size_t)sg.frame * kmax * 2;
    const float* ds = desc + (size_t)sg.frame * kmax * LG_D;
    for (int e = threadIdx.x; e < 64 * 16; e += 256) {
        const int i = r0 + e / 16, p = e % 16;
        const size_t r = (size_t)sg.off + i;
        const bool live = i < sg.len;
        float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);  // cos f, cos f + 1, sin f, sin f + 1
        if (live) {
            const float kx = (kp[2 * i] - nm.x) / nm.z, ky = (kp[2 * i + 1] - nm.y) / nm.z;
            const float p0 = kx * Wr[4 * p] + ky * Wr[4 * p + 1];
            const float p1 = kx * Wr[4 * p + 2] + ky * Wr[4 * p + 3];
            cs = make_float4(cosf(p0), cosf(p1), sinf(p0), sinf(p1));
        }
        efac[lg_fac4(r, p)] = cs;
        if (p == 0) ind[r] = live ? i : -1;
    }
    if (mv) {
        const size_t fo = (size_t)mv[blockIdx.y].z;
        for (int e = threadIdx.x; e < 64 * LG_D / 4; e += 256) {
            const int i = r0 + e / (LG_D / 4), c4 = (e % (LG_D / 4)) * 4;
            const size_t r = (size_t)sg.off + i;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            uint2 o = make_uint2(0u, 0u);
            if (i < sg.len) {
                v = *reinterpret_cast<const float4*>(xf + (fo + i) * LG_D + c4);
                o = *reinterpret_cast<const uint2*>(catf + (fo + i) * 512 + c4);
            }
            *reinterpret_cast<float4*>(x + r * LG_D + c4) = v;
            *reinterpret_cast<uint2*>(cat + r * 512 + c4) = o;
        }
        return;
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
                                                    const float* __restrict__ x, const float4* __restrict__ efac,
                                                    const int32_t* __restrict__ ind,
                                                    float* __restrict__ x2, bf16_t* __restrict__ cat2,
                                                    float4* __restrict__ efac2,
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
    // 16-B x loads / stores and 8-B bf16 stores per lane (the same RNE conversion per
    // element as f32_to_bf16); a wave moves one whole 1 KiB row of x per instruction
    for (int e = tid; e < mv.y * (LG_D / 4); e += 256) {
        const int i = e / (LG_D / 4), c4 = (e % (LG_D / 4)) * 4;
        const int rk = rank[i];
        if (rk < 0) continue;
        const float4 val = *reinterpret_cast<const float4*>(x + (size_t)(mv.x + i) * LG_D + c4);
        *reinterpret_cast<float4*>(x2 + (size_t)(mv.z + rk) * LG_D + c4) = val;
        *reinterpret_cast<uint2*>(cat2 + (size_t)(mv.z + rk) * 512 + c4) =
            make_uint2(pack_bf16x2(val.x, val.y), pack_bf16x2(val.z, val.w));
    }
    for (int e = tid; e < mv.y * 16; e += 256) {
        const int i = e / 16, p = e % 16;
        const int rk = rank[i];
        if (rk < 0) continue;
        efac2[lg_fac4((size_t)(mv.z + rk), p)] = efac[lg_fac4((size_t)(mv.x + i), p)];
    }
    for (int i = tid; i < mv.y; i += 256)
        if (rank[i] >= 0) ind2[mv.z + rank[i]] = ind[mv.x + i];
    // zero the padding rows of the new segment
    for (int e = tid; e < (padded - newlen) * (LG_D / 4); e += 256) {
        const int i = newlen + e / (LG_D / 4), c4 = (e % (LG_D / 4)) * 4;
        *reinterpret_cast<float4*>(x2 + (size_t)(mv.z + i) * LG_D + c4) = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<uint2*>(cat2 + (size_t)(mv.z + i) * 512 + c4) = make_uint2(0u, 0u);
    }
    for (int e = tid; e < (padded - newlen) * 16; e += 256) {
        const int i = newlen + e / 16, p = e % 16;
        efac2[lg_fac4((size_t)(mv.z + i), p)] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int i = newlen + tid; i < padded; i += 256) ind2[mv.z + i] = -1;
}

__global__ void k_lg_live(const Seg* __restrict__ segs, int nseg, uint8_t* __restrict__ live,
                          int* __restrict__ rowseg, int Npad) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= Npad) return;
    // segments are in increasing offset order: binary search for the last one starting
    // at or before r (a linear scan over every segment per row was quadratic)
    int lo = 0, hi = nseg - 1, sgi = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (segs[mid].off <= r) {
            sgi = mid;
            lo = mid + 1;
        } else {
            hi = mid - 1;
        }
    }
    if (sgi >= 0 && r >= segs[sgi].off + segs[sgi].len) sgi = -1;
    live[r] = sgi >= 0;
    rowseg[r] = sgi;
}

// ------------------------------------------------------------------ assignment
// For every finishing pair a (table entry Asg): S = final_proj(x0) . final_proj(x1)^T
// (the two 1/4 scales applied here as one exact 1/16), the row / column log_softmax
// terms (torch form (x - max) - log(sum exp(x - max))), and the row / column argmax of
// (s0 + s1) + (lz0 + lz1)  (first index on ties, as torch.max), then the mutual filter.
// Row / column statistics are indexed by layout row, so all pairs share the buffers.
// Tile grids carry the pair in blockIdx.z, line grids in blockIdx.y.
//
//   k_asg_sim      128 x 128 GEMM tile -> S (whole float4 rows) + the tile's partial
//                  (max, sum exp) of every row and column, from the LDS-staged tile;
//   k_asg_stats    combines the partials -> row / column (max, log sum exp);
//   k_asg_arg      reads each 64 x 128 tile of S once -> per-tile best (score, index)
//                  of every row and column;
//   k_asg_argfinal combines them -> row argmax + value, column argmax.
// S is written once and read once.
struct Asg {
    int m, n, ra, rb;  // rows of image a / b, their first layout rows
    long soff;         // S offset (floats)
    int pair, ld;      // pair index, S row stride (n rounded up to 4: float4 rows)
    int lo_first, pad; // image a's frame index > image b's: k_asg_sim's cross-term order
};

constexpr int SBM = 128;               // k_asg_sim tile (rows = columns)
constexpr int TSS = SBM + 4;           // its LDS row stride: the 16 lanes of a b128 group (16 rows)
                                       // and the 64 lanes of a b32 column read hit distinct banks
constexpr int ARM = 64, ARN = 128;     // k_asg_arg tile
#ifndef MLG_ASG_FULL
#define MLG_ASG_FULL 1  // k_asg_arg: straight-line scans for full tiles (0: the general loops only, A/B)
#endif
constexpr int TSA = ARN + 8;           // its LDS row stride: b128 groups of 8 rows x 2 halves

// per-tile partials: part[((slot * 2 + dir) * tiles + t) * kmax + i]; dir 0 = rows
// (t = 128-column tile), dir 1 = columns (t = row tile: 128 rows in k_asg_sim's
// statistics, 64 in k_asg_arg's bests)
__device__ __forceinline__ size_t part_at(int slot, int dir, int t, int i, int kmax) {
    return ((size_t)(slot * 2 + dir) * ((kmax + ARM - 1) / ARM) + t) * kmax + i;
}

// S = MD[ra .. ra + m) . MD[rb .. rb + n)^T of every listed pair in ONE launch.  MD is
// final_proj(x) (f32 accumulate) held as bf16 hi + lo halves (hi = bf16(y), lo =
// bf16(y - hi), k-step-major [16][rows][16]; gemm_bf16.hip EpiBiasSplitBF16), and the
// product is hi.hi + hi.lo + lo.hi on v_mfma_f32_32x32x16_bf16 with f32 accumulation:
// operand error ~2^-17, dropped lo.lo ~2^-18 relative -- f32-class accuracy (upstream
// runs this einsum in float32) at 3 bf16 MFMAs instead of 8 exact-f32 32x32x2 ones per
// 16-deep k-step.  4 waves of 64 x 64; each wave streams its operand fragments straight
// from L2 (one contiguous 1 KiB per wave-load), double-buffered one k-step ahead.
#ifndef ASG_PF
#define ASG_PF 1
#endif
__global__ __launch_bounds__(256, 2) void k_asg_sim(const Asg* __restrict__ tab, const bf16_t* __restrict__ MDH,
                                                    const bf16_t* __restrict__ MDL, int rows,
                                                    float* __restrict__ Sall, float2* __restrict__ part, int kmax) {
    const Asg a = tab[blockIdx.z];
    const int m0 = blockIdx.y * SBM, n0 = blockIdx.x * SBM;
    if (m0 >= a.m || n0 >= a.n) return;
    __shared__ __attribute__((aligned(16))) float T[SBM * TSS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 31, hh = lane >> 5;
    const int wm = wave >> 1, wn = wave & 1;
    const size_t step = (size_t)rows * 16;
    size_t ao[2], bo[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
        ao[x] = (size_t)(a.ra + min(m0 + wm * 64 + 32 * x + col, a.m - 1)) * 16 + 8 * hh;
        bo[x] = (size_t)(a.rb + min(n0 + wn * 64 + 32 * x + col, a.n - 1)) * 16 + 8 * hh;
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.f;
    // ASG_PF k-steps of fragments in flight (2 = double buffer); each step's 8 loads are
    // L2 round trips that one step of 12 MFMAs does not cover
    constexpr int NB = ASG_PF + 1;
    bf16x8 ah[NB][2], al[NB][2], bh[NB][2], bl[NB][2];  // [buffer][x or y]
#pragma unroll
    for (int pf = 0; pf < ASG_PF; ++pf) {
        const size_t o = (size_t)pf * step;
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            ah[pf][x] = *reinterpret_cast<const bf16x8*>(MDH + o + ao[x]);
            al[pf][x] = *reinterpret_cast<const bf16x8*>(MDL + o + ao[x]);
            bh[pf][x] = *reinterpret_cast<const bf16x8*>(MDH + o + bo[x]);
            bl[pf][x] = *reinterpret_cast<const bf16x8*>(MDL + o + bo[x]);
        }
    }
#pragma unroll
    for (int ks = 0; ks < LG_D / 16; ++ks) {
        const int cb = ks % NB, nb = (ks + ASG_PF) % NB;
        if (ks + ASG_PF < LG_D / 16) {
            const size_t o = (size_t)(ks + ASG_PF) * step;
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                ah[nb][x] = *reinterpret_cast<const bf16x8*>(MDH + o + ao[x]);
                al[nb][x] = *reinterpret_cast<const bf16x8*>(MDL + o + ao[x]);
                bh[nb][x] = *reinterpret_cast<const bf16x8*>(MDH + o + bo[x]);
                bl[nb][x] = *reinterpret_cast<const bf16x8*>(MDL + o + bo[x]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // next step's loads stay ahead of this step's MFMAs
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
                // the two cross terms in a canonical order: hi of the lower frame's image x lo
                // of the other first, whichever side it is on.  The swapped call (b, a) then
                // adds the same products in the same order to every element, so S(b, a) is
                // S(a, b)^T bit for bit and LightGlue(b, a) is exactly swap(LightGlue(a, b))
                // -- what lets the full gate match each unordered pair once (pipeline.py).
                // (A fixed ah.bl-then-al.bh order rounded the swapped call's cross terms the
                // other way round: 1 of 1024 reverse pairs kept a different match, r02k.)
                if (!a.lo_first) {
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[cb][x], bl[cb][y], acc[x][y], 0, 0, 0);
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[cb][x], bh[cb][y], acc[x][y], 0, 0, 0);
                } else {
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[cb][x], bh[cb][y], acc[x][y], 0, 0, 0);
                    acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[cb][x], bl[cb][y], acc[x][y], 0, 0, 0);
                }
                acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[cb][x], bh[cb][y], acc[x][y], 0, 0, 0);
            }
    }
    // D[i][j]: col j = lane & 31, row i = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int j = wn * 64 + y * 32 + col;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                T[(wm * 64 + x * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh) * TSS + j] = acc[x][y][r];
        }
    __syncthreads();
    const int mr = min(SBM, a.m - m0), nc = min(SBM, a.n - n0);
    float* S = Sall + a.soff;
#pragma unroll 4
    for (int it = 0; it < SBM / 8; ++it) {
        // ld is a multiple of 4 and columns n .. ld are scratch: whole float4s while c < nc
        const int r = it * 8 + (tid >> 5), c = (tid & 31) * 4;
        if (r < mr && c < nc)
            *reinterpret_cast<float4*>(S + (size_t)(m0 + r) * a.ld + n0 + c) =
                *reinterpret_cast<const float4*>(T + r * TSS + c);
    }
    // partial softmax statistics: threads 0-127 one row each, 128-255 one column each;
    // exp(v / 16 - mx) as exp2 of one FMA (v_exp_f32)
    constexpr float L2E = 1.4426950408889634f;
    const bool colw = tid >= SBM;
    const int q = tid & (SBM - 1);
    if (q >= (colw ? nc : mr)) return;
    float mx = -INFINITY, sm = 0.f;
    if (MLG_ASG_FULL && (colw ? mr : nc) == SBM) {
        // full-length line: straight-line scans, no per-element bounds test (same order)
        if (colw) {
#pragma unroll 8
            for (int e = 0; e < SBM; ++e) mx = fmaxf(mx, T[e * TSS + q]);
            mx *= 0.0625f;
            const float nm = -mx * L2E;
#pragma unroll 8
            for (int e = 0; e < SBM; ++e) sm += __builtin_amdgcn_exp2f(fmaf(T[e * TSS + q], 0.0625f * L2E, nm));
        } else {
            const float* p = T + q * TSS;
#pragma unroll 8
            for (int e = 0; e < SBM; e += 4) {
                const float4 v = *reinterpret_cast<const float4*>(p + e);
                mx = fmaxf(mx, v.x);
                mx = fmaxf(mx, v.y);
                mx = fmaxf(mx, v.z);
                mx = fmaxf(mx, v.w);
            }
            mx *= 0.0625f;
            const float nm = -mx * L2E;
#pragma unroll 8
            for (int e = 0; e < SBM; e += 4) {
                const float4 v = *reinterpret_cast<const float4*>(p + e);
                sm += __builtin_amdgcn_exp2f(fmaf(v.x, 0.0625f * L2E, nm));
                sm += __builtin_amdgcn_exp2f(fmaf(v.y, 0.0625f * L2E, nm));
                sm += __builtin_amdgcn_exp2f(fmaf(v.z, 0.0625f * L2E, nm));
                sm += __builtin_amdgcn_exp2f(fmaf(v.w, 0.0625f * L2E, nm));
            }
        }
    } else if (colw) {
        for (int e = 0; e < mr; ++e) mx = fmaxf(mx, T[e * TSS + q]);
        mx *= 0.0625f;
        const float nm = -mx * L2E;
        for (int e = 0; e < mr; ++e) sm += __builtin_amdgcn_exp2f(fmaf(T[e * TSS + q], 0.0625f * L2E, nm));
    } else {
        const float* p = T + q * TSS;
        for (int e = 0; e < nc; e += 4) {
            const float4 v = *reinterpret_cast<const float4*>(p + e);
            mx = fmaxf(mx, v.x);
            if (e + 1 < nc) mx = fmaxf(mx, v.y);
            if (e + 2 < nc) mx = fmaxf(mx, v.z);
            if (e + 3 < nc) mx = fmaxf(mx, v.w);
        }
        mx *= 0.0625f;
        const float nm = -mx * L2E;
        for (int e = 0; e < nc; e += 4) {
            const float4 v = *reinterpret_cast<const float4*>(p + e);
            sm += __builtin_amdgcn_exp2f(fmaf(v.x, 0.0625f * L2E, nm));
            if (e + 1 < nc) sm += __builtin_amdgcn_exp2f(fmaf(v.y, 0.0625f * L2E, nm));
            if (e + 2 < nc) sm += __builtin_amdgcn_exp2f(fmaf(v.z, 0.0625f * L2E, nm));
            if (e + 3 < nc) sm += __builtin_amdgcn_exp2f(fmaf(v.w, 0.0625f * L2E, nm));
        }
    }
    part[colw ? part_at(blockIdx.z, 1, blockIdx.y, n0 + q, kmax) : part_at(blockIdx.z, 0, blockIdx.x, m0 + q, kmax)] =
        make_float2(mx, sm);
}

// row / column (max, log sum exp) from k_asg_sim's partials; grid (.., pairs, 2 dirs)
__global__ __launch_bounds__(256) void k_asg_stats(const Asg* __restrict__ tab, const float2* __restrict__ part,
                                                   int kmax, float* __restrict__ rmax, float* __restrict__ rlog,
                                                   float* __restrict__ cmax, float* __restrict__ clog) {
    const Asg a = tab[blockIdx.y];
    const int dir = blockIdx.z;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= (dir ? a.n : a.m)) return;
    const int nt = ((dir ? a.m : a.n) + SBM - 1) / SBM;
    const float2* p = part + part_at(blockIdx.y, dir, 0, i, kmax);
    float M = -INFINITY;
    for (int t = 0; t < nt; ++t) M = fmaxf(M, p[(size_t)t * kmax].x);
    float S = 0.f;
    for (int t = 0; t < nt; ++t) S += p[(size_t)t * kmax].y * expf(p[(size_t)t * kmax].x - M);
    const int o = dir ? a.rb + i : a.ra + i;
    (dir ? cmax : rmax)[o] = M;
    (dir ? clog : rlog)[o] = logf(S);
}

__device__ __forceinline__ float lg_score(float v, float rm, float rl, float cm, float cl, float cert) {
    return (((v - rm) - rl) + ((v - cm) - cl)) + cert;
}

// (score, index) a beats b: higher score, the lower index on ties
__device__ __forceinline__ bool beats(float sa, int ia, float sb, int ib) { return sa > sb || (sa == sb && ia < ib); }

// per-tile best (score, index) of every row and column of a 64 x 128 tile of S (4 tiles
// in flight per CU so the HBM read of one overlaps the scoring of another): threads
// 0-127 two per row (alternate float4 column chunks, combined by one shuffle), 128-255
// one per column; each scans increasing indices with strict >, keeping the first index
__global__ __launch_bounds__(256, 4) void k_asg_arg(const Asg* __restrict__ tab, const float* __restrict__ Sall,
                                                    const float* __restrict__ rmax, const float* __restrict__ rlog,
                                                    const float* __restrict__ cmax, const float* __restrict__ clog,
                                                    const float* __restrict__ lz, float2* __restrict__ part, int kmax) {
    const Asg a = tab[blockIdx.z];
    const int m0 = blockIdx.y * ARM, n0 = blockIdx.x * ARN;
    if (m0 >= a.m || n0 >= a.n) return;
    __shared__ __attribute__((aligned(16))) float T[ARM * TSA];
    __shared__ float4 sr[ARM], sc[ARN];  // (max, log sum, log-sigmoid) of the tile's rows / columns
    const int tid = threadIdx.x;
    const int mr = min(ARM, a.m - m0), nc = min(ARN, a.n - n0);
    const float* S = Sall + a.soff;
#pragma unroll
    for (int it = 0; it < ARM / 8; ++it) {
        const int r = it * 8 + (tid >> 5), c = (tid & 31) * 4;
        if (r < mr && c < nc)
            *reinterpret_cast<float4*>(T + r * TSA + c) =
                *reinterpret_cast<const float4*>(S + (size_t)(m0 + r) * a.ld + n0 + c);
    }
    if (tid < ARM) {
        if (tid < mr) {
            const int o = a.ra + m0 + tid;
            sr[tid] = make_float4(rmax[o], rlog[o], lz[o], 0.f);
        }
    } else if (tid >= ARN) {
        const int j = tid - ARN;
        if (j < nc) {
            const int o = a.rb + n0 + j;
            sc[j] = make_float4(cmax[o], clog[o], lz[o], 0.f);
        }
    }
    __syncthreads();
    float best = -INFINITY;
    int bi = 0x7fffffff;
    if (tid < ARN) {
        const int r = tid >> 1, h = tid & 1;
        if (r < mr && MLG_ASG_FULL && nc == ARN) {
            // full-width tile: straight-line scan, no per-element bounds test (same scores,
            // same order, same strict > -- the general loop below, branch-free)
            const float4 me = sr[r];
            const float* p = T + r * TSA;
#pragma unroll 4
            for (int q = 0; q < ARN / 8; ++q) {
                const int c = 8 * q + 4 * h;
                const float4 v = *reinterpret_cast<const float4*>(p + c);
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float4 ot = sc[c + k];
                    const float s = lg_score(vv[k] * 0.0625f, me.x, me.y, ot.x, ot.y, me.z + ot.z);
                    const bool g = s > best;
                    best = g ? s : best;
                    bi = g ? c + k : bi;
                }
            }
        } else if (r < mr) {
            const float4 me = sr[r];
            const float* p = T + r * TSA;
            for (int c = 4 * h; c < nc; c += 8) {
                const float4 v = *reinterpret_cast<const float4*>(p + c);
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (c + k >= nc) break;
                    const float4 ot = sc[c + k];
                    const float s = lg_score(vv[k] * 0.0625f, me.x, me.y, ot.x, ot.y, me.z + ot.z);
                    if (s > best) {
                        best = s;
                        bi = c + k;
                    }
                }
            }
        }
        const float ob = __shfl_xor(best, 1, 64);
        const int oi = __shfl_xor(bi, 1, 64);
        if (beats(ob, oi, best, bi)) {
            best = ob;
            bi = oi;
        }
        if (h == 0 && r < mr)
            part[part_at(blockIdx.z, 0, blockIdx.x, m0 + r, kmax)] =
                make_float2(best, __int_as_float(bi == 0x7fffffff ? bi : n0 + bi));
    } else {
        const int j = tid - ARN;
        if (j >= nc) return;
        const float4 me = sc[j];
        if (MLG_ASG_FULL && mr == ARM) {
#pragma unroll 8
            for (int e = 0; e < ARM; ++e) {
                const float4 ot = sr[e];
                const float s = lg_score(T[e * TSA + j] * 0.0625f, ot.x, ot.y, me.x, me.y, ot.z + me.z);
                const bool g = s > best;
                best = g ? s : best;
                bi = g ? e : bi;
            }
        } else {
            for (int e = 0; e < mr; ++e) {
                const float4 ot = sr[e];
                const float s = lg_score(T[e * TSA + j] * 0.0625f, ot.x, ot.y, me.x, me.y, ot.z + me.z);
                if (s > best) {
                    best = s;
                    bi = e;
                }
            }
        }
        part[part_at(blockIdx.z, 1, blockIdx.y, n0 + j, kmax)] =
            make_float2(best, __int_as_float(bi == 0x7fffffff ? bi : m0 + bi));
    }
}

// row argmax + value, column argmax from the per-tile bests (tiles in increasing index
// order, strict >: the first index on ties); grid (.., pairs, 2 dirs).  A line with no
// finite score (NaN input) points at index 0 with value -inf.
__global__ __launch_bounds__(256) void k_asg_argfinal(const Asg* __restrict__ tab, const float2* __restrict__ part,
                                                      int kmax, int* __restrict__ arg, float* __restrict__ val) {
    const Asg a = tab[blockIdx.y];
    const int dir = blockIdx.z;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= (dir ? a.n : a.m)) return;
    const int nt = dir ? (a.m + ARM - 1) / ARM : (a.n + ARN - 1) / ARN;
    const float2* p = part + part_at(blockIdx.y, dir, 0, i, kmax);
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int t = 0; t < nt; ++t) {
        const float2 c = p[(size_t)t * kmax];
        if (c.x > best) {
            best = c.x;
            bi = __float_as_int(c.y);
        }
    }
    if (bi == 0x7fffffff) {
        bi = 0;
        best = -INFINITY;
    }
    if (dir) {
        arg[a.rb + i] = bi;
    } else {
        arg[a.ra + i] = bi;
        val[a.ra + i] = best;
    }
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


// ---------------------------------------------------------- pair orientation
// Ordered pair p takes the matches of unordered-pair row rows[p]; with swap[p] the
// image roles are exchanged: (i0, i1) -> (i1, i0), re-sorted ascending in the new image0
// index, which is the order LightGlue itself returns for the swapped call (its matches
// are mutual nearest neighbours, so each index appears at most once: a scatter into
// kmax slots plus an ordered compaction sorts them exactly).  Scores follow their match.
__global__ __launch_bounds__(256) void k_lg_orient(const int32_t* __restrict__ m_in, const float* __restrict__ s_in,
                                                   const int32_t* __restrict__ n_in, const int32_t* __restrict__ rows,
                                                   const uint8_t* __restrict__ swap, int kmax,
                                                   int32_t* __restrict__ m_out, float* __restrict__ s_out,
                                                   int32_t* __restrict__ n_out) {
    __shared__ int slot[2048];
    __shared__ int wsum[256];
    const int p = blockIdx.x, tid = threadIdx.x, r = rows[p];
    const int n = n_in[r];
    const int32_t* mi = m_in + (size_t)r * kmax * 2;
    const float* si = s_in + (size_t)r * kmax;
    int32_t* mo = m_out + (size_t)p * kmax * 2;
    float* so = s_out + (size_t)p * kmax;
    if (!swap[p]) {
        for (int i = tid; i < n; i += 256) {
            mo[2 * i] = mi[2 * i];
            mo[2 * i + 1] = mi[2 * i + 1];
            so[i] = si[i];
        }
        if (tid == 0) n_out[p] = n;
        return;
    }
    for (int i = tid; i < kmax; i += 256) slot[i] = -1;
    __syncthreads();
    for (int i = tid; i < n; i += 256) slot[mi[2 * i + 1]] = i;  // image1 index -> match
    __syncthreads();
    const int per = (kmax + 255) / 256, b0 = tid * per;  // ordered compaction of the slots
    int c = 0;
    for (int j = b0; j < min(b0 + per, kmax); ++j) c += slot[j] >= 0;
    wsum[tid] = c;
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int t = 0; t < 256; ++t) { const int v = wsum[t]; wsum[t] = acc; acc += v; }
    }
    __syncthreads();
    int o = wsum[tid];
    for (int j = b0; j < min(b0 + per, kmax); ++j) {
        const int i = slot[j];
        if (i < 0) continue;
        mo[2 * o] = j;
        mo[2 * o + 1] = mi[2 * i];
        so[o] = si[i];
        ++o;
    }
    if (tid == 0) n_out[p] = n;
}


#if !MLG_LG_INIT_FUSED
// Layer 0's self block on the frame layout -> the pair layout: pair segment k copies the
// rows of its frame's segment (x f32 and the bf16 x copy in CAT's first 256 columns).
// mv[k] = (pair offset, live rows, frame offset, -).
__global__ __launch_bounds__(256) void k_lg_gather_rows(const int4* __restrict__ mv, const float* __restrict__ xf,
                                                        const bf16_t* __restrict__ catf, float* __restrict__ x,
                                                        bf16_t* __restrict__ cat) {
    const int4 m = mv[blockIdx.y];
    const int r0 = blockIdx.x * 16;
    if (r0 >= m.y) return;
    for (int e = threadIdx.x; e < 16 * 64; e += 256) {  // 16 rows x 64 float4 of x
        const int i = r0 + e / 64, c = e % 64;
        if (i >= m.y) continue;
        reinterpret_cast<float4*>(x + (size_t)(m.x + i) * LG_D)[c] =
            reinterpret_cast<const float4*>(xf + (size_t)(m.z + i) * LG_D)[c];
    }
    for (int e = threadIdx.x; e < 16 * 32; e += 256) {  // 16 rows x 32 x 16 B of the bf16 copy
        const int i = r0 + e / 32, c = e % 32;
        if (i >= m.y) continue;
        reinterpret_cast<uint4*>(cat + (size_t)(m.x + i) * 512)[c] =
            reinterpret_cast<const uint4*>(catf + (size_t)(m.z + i) * 512)[c];
    }
}
#endif

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

// ------------------------------------------------------------------ debug trace
// mlg_dbg_lg_trace_begin / _end (include/mlgate.h): the calling thread's mlg_lightglue
// calls append, after every stage, one 64-bit hash per 64-row tile of the buffer the
// stage wrote (planes x tiles of tile_bytes), so two runs can be compared stage by stage.
struct LgTrace {
    uint64_t* buf = nullptr;
    size_t cap = 0, used = 0;
    bool overflow = false;
    std::vector<int> tags, counts;
};
thread_local LgTrace* t_trace = nullptr;

// tile t = rows [t * rpt, (t + 1) * rpt) of each plane; row r's first row_bytes bytes
// (a multiple of 4) at base + plane * plane_stride + r * row_stride; rows with
// live[r] == 0 skipped when `live` is given (padding rows hold stale workspace)
__global__ __launch_bounds__(256) void k_dbg_hash(const uint8_t* __restrict__ base, int rpt, int row_bytes,
                                                  size_t row_stride, int planes, size_t plane_stride,
                                                  const uint8_t* __restrict__ live, uint64_t* __restrict__ out) {
    const int wpr = row_bytes / 4, words = rpt * wpr;
    uint64_t h = 0;
    for (int p = 0; p < planes; ++p)
        for (int i = threadIdx.x; i < words; i += 256) {
            const size_t r = (size_t)blockIdx.x * rpt + i / wpr;
            if (live && !live[r]) continue;
            uint64_t w = *reinterpret_cast<const uint32_t*>(base + p * plane_stride + r * row_stride + (i % wpr) * 4);
            w ^= (uint64_t)((size_t)p * words + i + 1) * 0x9E3779B97F4A7C15ull;
            w ^= w >> 33;
            w *= 0xff51afd7ed558ccdull;
            w ^= w >> 33;
            w *= 0xc4ceb9fe1a85ec53ull;
            w ^= w >> 33;
            h += w;
        }
    __shared__ uint64_t sh[256];
    sh[threadIdx.x] = h;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}

// tag = layer * 100 + stage (layer 99: layer 0's self block on the frame layout)
void trace(int tag, const void* base, int rpt, int row_bytes, size_t row_stride, int planes, size_t plane_stride,
           int ntiles, hipStream_t s, const uint8_t* live = nullptr) {
    LgTrace* t = t_trace;
    if (!t || ntiles <= 0 || row_bytes < 4) return;
    if (t->used + (size_t)ntiles > t->cap) {
        t->overflow = true;
        return;
    }
    hipLaunchKernelGGL(k_dbg_hash, dim3((unsigned)ntiles), dim3(256), 0, s, (const uint8_t*)base, rpt, row_bytes & ~3,
                       row_stride, planes, plane_stride, live, t->buf + t->used);
    t->used += ntiles;
    t->tags.push_back(tag);
    t->counts.push_back(ntiles);
}

struct LgLayout {
    size_t x, cat, efac, ind, x2, cat2, efac2, ind2, Q, K, Vt, ctx, hf, hb, live, rowseg, lz, keep,
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
    L.efac = take(N * 64 * 4);  // rotary factors, lg_fac4 layout
    L.ind = take(N * 4);
    L.x2 = take(N * LG_D * 4);
    L.cat2 = take(N * 512 * 2);
    L.efac2 = take(N * 64 * 4);
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
    L.part = take((size_t)L.asg_cap * 2 * ((kmax + ARM - 1) / ARM) * kmax * sizeof(float2));
    L.asg = take((size_t)P * sizeof(Asg));
    L.norm = take((size_t)2 * P * sizeof(float4));
    L.S = take((size_t)L.asg_cap * kmax * ((kmax + 3) & ~3) * 4);
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
    float4* EF = (float4*)(base + L.efac);
    int32_t* IND = (int32_t*)(base + L.ind);
    float* X2 = (float*)(base + L.x2);
    bf16_t* CAT2 = (bf16_t*)(base + L.cat2);
    float4* EF2 = (float4*)(base + L.efac2);
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
    bf16_t* MDH = (bf16_t*)(base + L.mdesc);  // hi half, then the lo half
    float* RMAX = (float*)(base + L.rmax);
    float* RLOG = (float*)(base + L.rlog);
    float* CMAX = (float*)(base + L.cmax);
    float* CLOG = (float*)(base + L.clog);
    int* ARG = (int*)(base + L.arg);
    float* VAL = (float*)(base + L.val);
    float2* PART = (float2*)(base + L.part);
    Asg* ASG = (Asg*)(base + L.asg);
    float* SS = (float*)(base + L.S);
    // debug trace (mlg_dbg_lg_trace_begin): per-stage hashes of 64-row tiles
    // live rows only (LIVE is the current layout's mask); byte-per-row buffers as 64-B tiles
    auto tr_rows = [&](int tag, const void* p, size_t row_bytes, int np, size_t stride = 0) {
        if (!t_trace) return;
        if (row_bytes < 4) trace(tag, p, 1, 64, 64, 1, 0, np / 64, s);
        else trace(tag, p, 64, (int)row_bytes, stride ? stride : row_bytes, 1, 0, np / 64, s, LIVE);
    };
    auto tr_heads = [&](int tag, const void* p, int np) {  // Q / K / V^T: [4 heads][np rows][64] bf16
        if (t_trace) trace(tag, p, 64, 128, 128, 4, (size_t)np * 128, np / 64, s);
    };
    auto tr_tab = [&](int tag, const void* p, size_t bytes) {
        if (t_trace && bytes >= 4) trace(tag, p, 1, (int)bytes, 0, 1, 0, 1, s);
    };
    int tl = 0;  // layer of the next table upload (trace tags)

    // Host tables below are uploaded with hipMemcpyAsync on `s` and only rewritten after
    // the stream has been synchronised (the per-layer statistics read-back, and one final
    // synchronisation before returning), so the pageable sources outlive every copy that
    // reads them.
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
        tr_tab(tl * 100 + 3, SEGS, segs.size() * sizeof(Seg));
        tr_tab(tl * 100 + 4, TASKS, h_tasks.size() * sizeof(int4));
        tr_tab(tl * 100 + 5, OUTOFF, h_out.size() * sizeof(int));
        tr_rows(tl * 100 + 6, LIVE, 1, Npad);
        return MLG_OK;
    };
    // Layer 0's self block reads one image only (its tokens, its positional encoding), so
    // it runs once per distinct frame of the call -- a frame layout in the secondary
    // buffers -- and its output rows are copied into every pair segment of that frame:
    // the same kernels on the same rows, so the same bits as running it per pair.
    std::vector<Seg> fsegs;
    std::vector<int4> f_tasks, f_moves;
    std::vector<int> f_out;
    bool self0_done = false;
    {
        std::unordered_map<int, int> fidx;
        std::vector<int> fmap(segs.size());
        int foff = 0;
        for (size_t k = 0; k < segs.size(); ++k) {
            auto it = fidx.find(segs[k].frame);
            if (it == fidx.end()) {
                it = fidx.emplace(segs[k].frame, (int)fsegs.size()).first;
                fsegs.push_back(Seg{foff, segs[k].len, segs[k].frame, 0});
                foff += (segs[k].len + 63) & ~63;
            }
            fmap[k] = it->second;
        }
        if (fsegs.size() < segs.size()) {
            const int NpadF = std::max(foff, 64);
            int maxqf = 0;
            double tok = 0, work = 0;
            for (const Seg& f : fsegs) {
                f_tasks.push_back(make_int4(f.off, f.len, f.off, f.len));
                f_out.push_back(f.off);
                maxqf = std::max(maxqf, f.len);
                tok += f.len;
                work += 4.0 * LG_H * 64 * (double)f.len * f.len;
            }
            for (size_t k = 0; k < segs.size(); ++k)
                f_moves.push_back(make_int4(segs[k].off, segs[k].len, fsegs[fmap[k]].off, 0));
            const int nf = (int)fsegs.size();
            if (hipMemcpyAsync(SEGS, fsegs.data(), fsegs.size() * sizeof(Seg), hipMemcpyHostToDevice, s) != hipSuccess ||
                hipMemcpyAsync(TASKS, f_tasks.data(), f_tasks.size() * sizeof(int4), hipMemcpyHostToDevice, s) !=
                    hipSuccess ||
                hipMemcpyAsync(OUTOFF, f_out.data(), f_out.size() * sizeof(int), hipMemcpyHostToDevice, s) !=
                    hipSuccess ||
                hipMemcpyAsync(MOVES, f_moves.data(), f_moves.size() * sizeof(int4), hipMemcpyHostToDevice, s) !=
                    hipSuccess)
                return MLG_EHIP;
            hipLaunchKernelGGL(k_lg_live, dim3((NpadF + 255) / 256), dim3(256), 0, s, SEGS, nf, LIVE, ROWSEG, NpadF);
            hipLaunchKernelGGL(k_lg_kpnorm, dim3((unsigned)nf), dim3(256), 0, s, SEGS, kpts, kmax,
                               (float4*)(base + L.norm));
            hipLaunchKernelGGL(k_lg_init, dim3((unsigned)((kmax + 63) / 64), (unsigned)nf), dim3(256), 0, s, SEGS,
                               (const float4*)(base + L.norm), kpts, desc, kmax, w.Wr, X2, CAT2, EF2, IND2);
            MLG_LAUNCH_CHECK();
            tr_tab(9903, SEGS, fsegs.size() * sizeof(Seg));
            tr_tab(9904, TASKS, f_tasks.size() * sizeof(int4));
            tr_rows(9901, X2, LG_D * 4, NpadF);
            tr_rows(9902, CAT2, 512, NpadF, 1024);
            {
                MlgProfScope prof(6, s, 2.0 * tok * 768 * 256);
                LG_TRY(mlg_lg_proj(true, CAT2, 512, w.self[0].Wqkv, w.self[0].bqkv, (const float*)EF2, LIVE, Q, K, VT, NpadF, s));
            }
            tr_heads(9910, Q, NpadF);
            tr_heads(9911, K, NpadF);
            tr_heads(9912, VT, NpadF);
            {
                MlgProfScope prof(5, s, work);
                LG_TRY(mlg_attention_varlen(Q, K, VT, CTX, LG_D, NpadF, LG_H, TASKS, OUTOFF, nf, maxqf, s));
            }
            tr_rows(9913, CTX, 512, NpadF);
            {
                MlgProfScope prof(8, s, 917504.0 * tok);
                LG_TRY(mlg_lg_ffn(CTX, X2, CAT2, 512, NpadF, w.self[0], s, nullptr));
            }
            tr_rows(9914, X2, LG_D * 4, NpadF);
            tr_rows(9915, CAT2, 512, NpadF, 1024);
            self0_done = true;
        }
    }
    LG_TRY(upload_layout());
    hipLaunchKernelGGL(k_lg_kpnorm, dim3((unsigned)segs.size()), dim3(256), 0, s, SEGS, kpts, kmax, (float4*)(base + L.norm));
#if MLG_LG_INIT_FUSED
    hipLaunchKernelGGL(k_lg_init, dim3((unsigned)((kmax + 63) / 64), (unsigned)segs.size()), dim3(256), 0, s, SEGS,
                       (const float4*)(base + L.norm), kpts, desc, kmax, w.Wr, X, CAT, EF, IND,
                       self0_done ? (const int4*)MOVES : nullptr, X2, CAT2);
    MLG_LAUNCH_CHECK();
#else
    hipLaunchKernelGGL(k_lg_init, dim3((unsigned)((kmax + 63) / 64), (unsigned)segs.size()), dim3(256), 0, s, SEGS,
                       (const float4*)(base + L.norm), kpts, desc, kmax, w.Wr, X, CAT, EF, IND,
                       nullptr, nullptr, nullptr);
    MLG_LAUNCH_CHECK();
    if (self0_done) {
        hipLaunchKernelGGL(k_lg_gather_rows, dim3((unsigned)((kmax + 15) / 16), (unsigned)segs.size()), dim3(256), 0, s,
                           MOVES, X2, CAT2, X, CAT);
        MLG_LAUNCH_CHECK();
    }
#endif
    tr_rows(1, X, LG_D * 4, Npad);
    tr_rows(2, CAT, 512, Npad, 1024);

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
        // algorithmic FLOPs per live token: 2 (256 x 256 + 512 x 512 + 256 x 512) = 917,504.
        // Its HBM bytes per token (ctx + bf16 x in 512 + 512, f32 x read + written 1024 +
        // 1024, bf16 x copy 512 = 3,584) give 256 FLOP/B, near the ridge (2.5 PF / 8 TB/s =
        // 312): the three GEMM phases, not HBM, bound it, so the slot is
        // priced against the MFMA peak
        MlgProfScope prof(8, s, 917504.0 * live_tokens());
        return mlg_lg_ffn(CTX, X, CAT, 512, Npad, bw, s, conf);
    };
    // assignment + filter of the listed segment pairs (k = index of image a's segment)
    auto assign = [&](int i, const std::vector<size_t>& ks) -> int {
        // mdesc = final_proj(x) for every token, as bf16 hi + lo; the 1/4 per side folds into S / 16
        LG_TRY(mlg_gemm_bias_split_bf16(CAT, 512, w.Wfinal[i], w.bfinal[i], MDH, MDH + (size_t)Npad * LG_D, Npad, LG_D,
                                         LG_D, s));
        if (t_trace) trace(i * 100 + 40, MDH, 64, 32, 32, 32, (size_t)Npad * 32, Npad / 64, s);
        // one table upload for all chunks (the per-layer statistics read-back orders its
        // reuse), so chunks follow each other without a host round trip
        h_asg.clear();
        for (size_t c = 0; c < ks.size(); ++c) {
            const Seg sa = segs[ks[c]], sb = segs[ks[c] + 1];
            Asg a;
            a.m = sa.len;
            a.n = sb.len;
            a.ra = sa.off;
            a.rb = sb.off;
            a.soff = (long)(c % L.asg_cap) * kmax * ((kmax + 3) & ~3);
            a.pair = pair_of[ks[c] / 2];
            a.ld = (sb.len + 3) & ~3;
            a.lo_first = sa.frame > sb.frame;
            a.pad = 0;
            h_asg.push_back(a);
            if (stop_layer) stop_layer[a.pair] = i + 1;
        }
        if (hipMemcpyAsync(ASG, h_asg.data(), h_asg.size() * sizeof(Asg), hipMemcpyHostToDevice, s) != hipSuccess)
            return MLG_EHIP;
        tr_tab(i * 100 + 41, ASG, h_asg.size() * sizeof(Asg));
        for (size_t c0 = 0; c0 < ks.size(); c0 += L.asg_cap) {
            const size_t c1 = std::min(ks.size(), c0 + L.asg_cap);
            int maxm = 0, maxn = 0;
            for (size_t c = c0; c < c1; ++c) {
                maxm = std::max(maxm, h_asg[c].m);
                maxn = std::max(maxn, h_asg[c].n);
            }
            const unsigned na = (unsigned)(c1 - c0);
            const Asg* tab = ASG + c0;
            const dim3 stiles((maxn + SBM - 1) / SBM, (maxm + SBM - 1) / SBM, na),
                atiles((maxn + ARN - 1) / ARN, (maxm + ARM - 1) / ARM, na),
                lines((std::max(maxm, maxn) + 255) / 256, na, 2);
            hipLaunchKernelGGL(k_asg_sim, stiles, dim3(256), 0, s, tab, MDH, MDH + (size_t)Npad * LG_D, Npad, SS, PART,
                               kmax);
            hipLaunchKernelGGL(k_asg_stats, lines, dim3(256), 0, s, tab, PART, kmax, RMAX, RLOG, CMAX, CLOG);
            hipLaunchKernelGGL(k_asg_arg, atiles, dim3(256), 0, s, tab, SS, RMAX, RLOG, CMAX, CLOG, LZ, PART, kmax);
            hipLaunchKernelGGL(k_asg_argfinal, lines, dim3(256), 0, s, tab, PART, kmax, ARG, VAL);
            hipLaunchKernelGGL(k_lg_filter, dim3(na), dim3(256), 0, s, tab, ARG, VAL, IND, filter_thr, kmax, matches,
                               mscores, nmatch);
            MLG_LAUNCH_CHECK();
        }
        return MLG_OK;
    };

    std::vector<int> stats(segs.size() * 2);
    for (int i = 0; i < LG_L && !segs.empty(); ++i) {
        // self block: projection + rotary + head split fused in the GEMM epilogue (layer 0's
        // already ran per frame above when frames repeat)
        if (!(i == 0 && self0_done)) {
            {
                MlgProfScope prof(6, s, 2.0 * live_tokens() * 768 * 256);
                LG_TRY(mlg_lg_proj(true, CAT, 512, w.self[i].Wqkv, w.self[i].bqkv, (const float*)EF, LIVE, Q, K, VT, Npad, s));
            }
            tr_heads(i * 100 + 10, Q, Npad);
            tr_heads(i * 100 + 11, K, Npad);
            tr_heads(i * 100 + 12, VT, Npad);
            LG_TRY(attention(false));
            tr_rows(i * 100 + 13, CTX, 512, Npad);
            LG_TRY(ffn(w.self[i], nullptr));
            tr_rows(i * 100 + 14, X, LG_D * 4, Npad);
            tr_rows(i * 100 + 15, CAT, 512, Npad, 1024);
        }
        // cross block
        {
            MlgProfScope prof(6, s, 2.0 * live_tokens() * 512 * 256);
            LG_TRY(mlg_lg_proj(false, CAT, 512, w.cross[i].Wqkv, w.cross[i].bqkv, nullptr, LIVE, Q, nullptr, VT,
                               Npad, s));
        }
        tr_heads(i * 100 + 20, Q, Npad);
        tr_heads(i * 100 + 21, VT, Npad);
        LG_TRY(attention(true));
        tr_rows(i * 100 + 22, CTX, 512, Npad);
        // layer i's heads on the updated tokens: matchability log-sigmoid (the assignment's
        // certainty term) and, before the last layer, confidences + early-stop / prune flags
        const bool last = i == LG_L - 1;
        const mlg_lg_conf_i heads{ROWSEG, last ? nullptr : w.wconf[i], last ? nullptr : w.bconf[i], w.wmatch[i],
                                  w.bmatch[i], last ? 0.f : (depth_conf > 0.f ? conf_threshold(i) : -INFINITY),
                                  width_conf, LZ, KEEP};
        // (depth_confidence <= 0: upstream computes no token confidences, so its pruning
        // mask is matchability alone -- a threshold of -inf drops the "low confidence is
        // never pruned" term; the stop bit is unused then)
        LG_TRY(ffn(w.cross[i], &heads));
        tr_rows(i * 100 + 23, X, LG_D * 4, Npad);
        tr_rows(i * 100 + 24, CAT, 512, Npad, 1024);
        tr_rows(i * 100 + 25, LZ, 4, Npad);
        if (!last) tr_rows(i * 100 + 26, KEEP, 1, Npad);

        if (last) {
            std::vector<size_t> ks;
            for (size_t k = 0; k < segs.size(); k += 2) ks.push_back(k);
            LG_TRY(assign(i, ks));
            break;
        }
        hipLaunchKernelGGL(k_lg_segstats, dim3((unsigned)segs.size()), dim3(256), 0, s, SEGS, KEEP, STATS);
        MLG_LAUNCH_CHECK();
        tr_tab(i * 100 + 27, STATS, segs.size() * 2 * sizeof(int));
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
            hipLaunchKernelGGL(k_lg_compact, dim3((unsigned)h_moves.size()), dim3(256), 0, s, MOVES, KEEP, X, EF,
                               IND, X2, CAT2, EF2, IND2);
            MLG_LAUNCH_CHECK();
            std::swap(X, X2);
            std::swap(CAT, CAT2);
            std::swap(EF, EF2);
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
        tl = i + 1;
        if (!h_moves.empty()) tr_tab(tl * 100 + 31, MOVES, h_moves.size() * sizeof(int4));
        if (!segs.empty()) LG_TRY(upload_layout());
        if (!h_moves.empty() && !segs.empty()) tr_rows(tl * 100 + 30, X, LG_D * 4, Npad);
        stats.assign(segs.size() * 2, 0);
    }
    if (t_trace) {
        trace(9990, nmatch, 1, P * 4, 0, 1, 0, 1, s);
    }
    // the last assignment's table (h_asg) and possibly a final layout upload are pageable
    // copies still queued on s: they must complete before the vectors go out of scope
    if (hipStreamSynchronize(s) != hipSuccess) return MLG_EHIP;
    return MLG_OK;
}

int mlg_lg_orient_matches(const int32_t* matches, const float* scores, const int32_t* num_matches,
                          const int32_t* rows, const uint8_t* swap, int P, int kmax, int32_t* matches_out,
                          float* scores_out, int32_t* num_out, void* stream) {
    if (P <= 0) return MLG_OK;
    if (kmax <= 0 || kmax > 2048 || !matches || !scores || !num_matches || !rows || !swap || !matches_out ||
        !scores_out || !num_out)
        return MLG_EINVAL;
    hipLaunchKernelGGL(k_lg_orient, dim3((unsigned)P), dim3(256), 0, (hipStream_t)stream, matches, scores,
                       num_matches, rows, swap, kmax, matches_out, scores_out, num_out);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

// ---------------------------------------------------------------- debug trace ABI
extern "C" {
int mlg_dbg_lg_trace_begin(void* dev_buf, size_t bytes) {
    if (!dev_buf || bytes < 8) return MLG_EINVAL;
    delete t_trace;
    t_trace = new LgTrace;
    t_trace->buf = (uint64_t*)dev_buf;
    t_trace->cap = bytes / 8;
    return MLG_OK;
}

int mlg_dbg_lg_trace_end(int32_t* tags, int32_t* counts, int max_entries) {
    LgTrace* t = t_trace;
    if (!t) return MLG_EINVAL;
    t_trace = nullptr;
    const int n = (int)t->tags.size();
    const bool overflow = t->overflow;
    if (tags && counts)
        for (int i = 0; i < n && i < max_entries; ++i) {
            tags[i] = t->tags[i];
            counts[i] = t->counts[i];
        }
    delete t;
    return overflow ? MLG_ENOMEM : n;
}
}  // extern "C"
