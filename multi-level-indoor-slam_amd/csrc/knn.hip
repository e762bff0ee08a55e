// All-keyframes cosine kNN + time mask + threshold + floor gate (gfx950).
//
// Replaces SemanticPlaceRecognition.find_loop_closures (place_recognition.py:851-911)
// and compute_all_pairwise_similarities (:179-190):
//
//   k_row_normalize  Xn[i] = X[i] / (||X[i]||_2 + 1e-8) with the norm computed in
//                    numpy's exact float32 order (square, pairwise sum with 8-way
//                    unrolled <=128 leaves, 8192-element iterator chunks, sqrtf), so
//                    the normalised rows are bit-identical to the reference's.
//   k_sim_f32        S = Xn[q0:q1] . Xn^T with v_mfma_f32_32x32x2_f32 (exact f32 FMA
//                    chain; the reference's OpenBLAS SGEMM differs only in summation
//                    order).
//   k_topk_gate      per query row: drop |t_j - t_i| < min_gap (float64), top-k by
//                    (similarity desc, index desc), drop sim < thr, floor-consistency
//                    bit (gating && both labels present -> floor_i == floor_j), and
//                    integer totals of valid / rejected matches.
// Fused path (k <= 32, the default): no [Q, N] similarity matrix ever reaches HBM.
//   k_row_norm_wave  the same numpy-exact norm, one wave per row: the leaves of numpy's
//                    pairwise tree summed in parallel by lanes, combined in tree order.
//   k_knn_scan       64 query rows x one column split per workgroup: 64 x 128 tiles of
//                    S = Xn_q . Xn^T on the exact-f32 MFMA (the same k order as
//                    k_sim_f32, so the same bits), staged in LDS, and streamed into
//                    per-row top-k lists held across the lanes of a wave (lane l = rank
//                    l): a candidate that beats the row's k-th is inserted by one
//                    ballot + shuffle, so after the first tile almost every value is
//                    rejected by one compare.  Writes each row's sorted partial list.
//   k_knn_merge      per row: merges the column splits' lists, floor bit, totals.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {

// ---------------------------------------------------------------- norms -----
__device__ float pairwise_leaf(const float* a, int n) {
    if (n < 8) {
        float r = -0.0f;
        for (int i = 0; i < n; ++i) r = __fadd_rn(r, __fmul_rn(a[i], a[i]));
        return r;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = __fmul_rn(a[j], a[j]);
    int i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], __fmul_rn(a[i + j], a[i + j]));
    float res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                          __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
    for (; i < n; ++i) res = __fadd_rn(res, __fmul_rn(a[i], a[i]));
    return res;
}

// numpy pairwise_sum of squares, iteratively (post-order over the split tree).
__device__ float pairwise_sumsq(const float* a, int n) {
    int st_off[32], st_n[32], st_state[32];
    float st_val[32];
    int sp = 0;
    st_off[0] = 0; st_n[0] = n; st_state[0] = 0;
    float ret = 0.f;
    while (sp >= 0) {
        const int o = st_off[sp], m = st_n[sp];
        if (m <= 128) {
            ret = pairwise_leaf(a + o, m);
            --sp;
        } else {
            int n2 = m / 2;
            n2 -= n2 % 8;
            if (st_state[sp] == 0) {  // descend left
                st_state[sp] = 1;
                ++sp;
                st_off[sp] = o; st_n[sp] = n2; st_state[sp] = 0;
                continue;
            } else if (st_state[sp] == 1) {  // left done -> descend right
                st_val[sp] = ret;
                st_state[sp] = 2;
                ++sp;
                st_off[sp] = o + n2; st_n[sp] = m - n2; st_state[sp] = 0;
                continue;
            } else {
                ret = __fadd_rn(st_val[sp], ret);
                --sp;
            }
        }
        // propagate `ret` to the parent on the next loop iteration
    }
    return ret;
}

__global__ void k_row_normalize(const float* __restrict__ X, float* __restrict__ Xn, int N, int D, int ldx,
                                float* __restrict__ norms) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float* x = X + (size_t)i * ldx;
    float acc = 0.f;
    for (int c0 = 0; c0 < D; c0 += 8192) {
        const int n = min(8192, D - c0);
        const float p = pairwise_sumsq(x + c0, n);
        acc = c0 == 0 ? p : __fadd_rn(acc, p);
    }
    const float nrm = __fsqrt_rn(acc);
    if (norms) norms[i] = nrm;
    const float den = __fadd_rn(nrm, 1e-8f);
    float* y = Xn + (size_t)i * ldx;
    for (int j = 0; j < D; ++j) y[j] = __fdiv_rn(x[j], den);
}

// ------------------------------------------------------------ similarity ----
// 128 x 128 tile, BK = 16, 256 threads = 2 x 2 waves of 64 x 64 (2 x 2 MFMA 32x32).
constexpr int SBM = 128, SBN = 128, SBK = 16;

// The 128 x 128 tile (m0, n0) of A . B^T on the exact-f32 MFMA (rows of A past Q and of
// B past N are clamped copies: the caller masks them).  One k order for every caller, so
// k_sim_f32 and k_xcorr_tiles produce the same bits.
__device__ __forceinline__ void sim_tile(const float* __restrict__ A, int Q, const float* __restrict__ B, int N,
                                         int D, int m0, int n0, float (&As)[SBK][SBM + 4], float (&Bs)[SBK][SBN + 4],
                                         f32x16 (&acc)[2][2]) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    for (int k0 = 0; k0 < D; k0 += SBK) {
        // stage 128 rows x 16 k of each operand, transposed to [k][row]
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = tid + i * 256, row = c >> 2, kq = (c & 3) * 4;
            const int ar = min(m0 + row, Q - 1), br = min(n0 + row, N - 1);
            float ta[4], tb[4];
            if (k0 + kq + 3 < D) {
                const float4 va = *reinterpret_cast<const float4*>(A + (size_t)ar * D + k0 + kq);
                const float4 vb = *reinterpret_cast<const float4*>(B + (size_t)br * D + k0 + kq);
                ta[0] = va.x; ta[1] = va.y; ta[2] = va.z; ta[3] = va.w;
                tb[0] = vb.x; tb[1] = vb.y; tb[2] = vb.z; tb[3] = vb.w;
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool in = k0 + kq + u < D;
                    ta[u] = in ? A[(size_t)ar * D + k0 + kq + u] : 0.f;
                    tb[u] = in ? B[(size_t)br * D + k0 + kq + u] : 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) { As[kq + u][row] = ta[u]; Bs[kq + u][row] = tb[u]; }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < SBK; kk += 2) {
            const int k = kk + (lane >> 5);
            float a[2], b[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                a[t] = As[k][wm * 64 + t * 32 + (lane & 31)];
                b[t] = Bs[k][wn * 64 + t * 32 + (lane & 31)];
            }
#pragma unroll
            for (int ta = 0; ta < 2; ++ta)
#pragma unroll
                for (int tb = 0; tb < 2; ++tb)
                    acc[ta][tb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
        }
        __syncthreads();
    }
}

// St (optional): the transpose, St[j][i] = S[i][j] (SuperGlue's column passes)
// LFSIM: the stored value is LoFTR's coarse similarity (S / 256) / 0.1 (the reference
// scales each side by 1/16 and divides the product by the temperature 0.1), computed
// once here instead of in each dual-softmax pass over S (loftr.hip)
template <bool LFSIM = false>
__global__ __launch_bounds__(256, 2) void k_sim_f32(const float* __restrict__ A, int Q, const float* __restrict__ B,
                                                    int N, int D, float* __restrict__ S, int lds,
                                                    float* __restrict__ St, int ldt) {
    __shared__ float As[SBK][SBM + 4];
    __shared__ float Bs[SBK][SBN + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m0 = blockIdx.y * SBM, n0 = blockIdx.x * SBN;
    const int wm = wave >> 1, wn = wave & 1;
    f32x16 acc[2][2];
    sim_tile(A, Q, B, N, D, m0, n0, As, Bs, acc);
    if (LFSIM)
#pragma unroll
        for (int ta = 0; ta < 2; ++ta)
#pragma unroll
            for (int tb = 0; tb < 2; ++tb)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[ta][tb][r] = (acc[ta][tb][r] * (1.0f / 256.0f)) / 0.1f;
    // D[i][j]: col j = lane & 31, row i = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int ta = 0; ta < 2; ++ta)
#pragma unroll
        for (int tb = 0; tb < 2; ++tb) {
            const int j = n0 + wn * 64 + tb * 32 + (lane & 31);
            if (j >= N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = m0 + wm * 64 + ta * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (i < Q) S[(size_t)i * lds + j] = acc[ta][tb][r];
            }
            if (St) {  // 4 consecutive rows i per lane and r-group: one 16-B store into row j of St
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int i0 = m0 + wm * 64 + ta * 32 + 8 * g + 4 * (lane >> 5);
                    const f32x16& a = acc[ta][tb];
                    float* t = St + (size_t)j * ldt + i0;
                    if (i0 + 3 < Q) {
                        *reinterpret_cast<float4*>(t) = make_float4(a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]);
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (i0 + e < Q) t[e] = a[4 * g + e];
                    }
                }
            }
        }
}

// ----------------------------------------------------------- top-k + gate ---
__device__ __forceinline__ bool before(float va, int ia, float vb, int ib) {
    return va > vb || (va == vb && ia > ib);
}

// One wave per query row.  Each lane keeps a sorted list of its own best <= k
// candidates in LDS; the wave then merges the 64 lists k times by wave argmax.
// Query row r has time tq[r] / floor fq[r]; database column j has tdb[j] / fdb[j].
template <int KMAX>
__global__ __launch_bounds__(64) void k_topk_gate(const float* __restrict__ S, int lds, int N, int Q,
                                                  const double* __restrict__ tq, const double* __restrict__ tdb,
                                                  const int64_t* __restrict__ fq, const uint8_t* __restrict__ hfq,
                                                  const int64_t* __restrict__ fdb, const uint8_t* __restrict__ hfdb,
                                                  double min_gap, float thr, int k, int gating,
                                                  int32_t* __restrict__ idx_out, float* __restrict__ sim_out,
                                                  uint8_t* __restrict__ valid_out, int32_t* __restrict__ count_out,
                                                  unsigned long long* __restrict__ totals) {
    __shared__ float lv[64 * KMAX];
    __shared__ int li[64 * KMAX];
    const int lane = threadIdx.x, r = blockIdx.x;
    if (r >= Q) return;
    const double ti = tq[r];
    const float* row = S + (size_t)r * lds;
    float* mv = lv + lane * KMAX;
    int* mi = li + lane * KMAX;
    int cnt = 0;
    for (int j = lane; j < N; j += 64) {
        if (fabs(tdb[j] - ti) < min_gap) continue;
        const float v = row[j];
        if (cnt == k && !before(v, j, mv[k - 1], mi[k - 1])) continue;
        int p = cnt < k ? cnt++ : k - 1;
        while (p > 0 && before(v, j, mv[p - 1], mi[p - 1])) {
            mv[p] = mv[p - 1];
            mi[p] = mi[p - 1];
            --p;
        }
        mv[p] = v;
        mi[p] = j;
    }
    int ptr = 0, emitted = 0, nvalid = 0;
    const bool hf_i = gating && hfq[r] != 0;
    const int64_t fi = gating ? fq[r] : 0;
    for (int step = 0; step < k; ++step) {
        float bv = ptr < cnt ? mv[ptr] : -INFINITY;
        int bi = ptr < cnt ? mi[ptr] : -1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(bv, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (oi >= 0 && (bi < 0 || before(ov, oi, bv, bi))) { bv = ov; bi = oi; }
        }
        if (bi < 0 || bv < thr) break;  // exhausted, or everything left is below threshold
        if (ptr < cnt && mi[ptr] == bi) ++ptr;
        if (lane == 0) {
            bool ok = true;
            if (hf_i && hfdb[bi]) ok = fi == fdb[bi];
            idx_out[(size_t)r * k + emitted] = bi;
            sim_out[(size_t)r * k + emitted] = bv;
            if (valid_out) valid_out[(size_t)r * k + emitted] = ok;
            nvalid += ok;
        }
        ++emitted;
    }
    if (lane == 0) {
        count_out[r] = emitted;
        if (totals) {
            atomicAdd(totals + 0, (unsigned long long)nvalid);
            atomicAdd(totals + 1, (unsigned long long)(emitted - nvalid));
        }
    }
}


// Large k (k > 256, no upper limit: the reference's argsort()[:k] has none): one
// workgroup per query row.  Each candidate is the 64-bit key (orderable similarity << 32
// | index), whose descending order is exactly (similarity desc, index desc).  The ranks
// are emitted in windows of TOPK_LARGE: a radix select over eight 8-bit digits (MSB
// first, 256-bin LDS histograms, one pass over the row each) finds the window's last key
// among the keys below the previous window's, those keys are gathered into LDS and
// bitonic-sorted, then emitted with the threshold / floor rule of k_topk_gate; the next
// window starts below the last key emitted.  Emission stops at the first similarity
// under the threshold, so a large k costs windows only while candidates pass it.
constexpr int TOPK_LARGE = 4096;
__device__ __forceinline__ uint64_t knn_key(float v, int j) {
    uint32_t u = __float_as_uint(v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((uint64_t)u << 32) | (uint32_t)j;
}
__global__ __launch_bounds__(256) void k_topk_large(const float* __restrict__ S, int lds, int N, int Q,
                                                    const double* __restrict__ tq, const double* __restrict__ tdb,
                                                    const int64_t* __restrict__ fq, const uint8_t* __restrict__ hfq,
                                                    const int64_t* __restrict__ fdb, const uint8_t* __restrict__ hfdb,
                                                    double min_gap, float thr, int k, int gating,
                                                    int32_t* __restrict__ idx_out, float* __restrict__ sim_out,
                                                    uint8_t* __restrict__ valid_out, int32_t* __restrict__ count_out,
                                                    unsigned long long* __restrict__ totals) {
    __shared__ uint64_t keys[TOPK_LARGE];
    __shared__ int hist[256];
    __shared__ int s_total, s_n, s_emitted, s_nvalid, s_stop;
    __shared__ uint64_t s_prefix, s_upper;
    __shared__ int s_need;
    const int tid = threadIdx.x, r = blockIdx.x;
    if (r >= Q) return;
    const double ti = tq[r];
    const float* row = S + (size_t)r * lds;
    // candidates left after the time-gap mask
    if (tid == 0) {
        s_total = 0;
        s_emitted = 0;
        s_nvalid = 0;
        s_stop = 0;
        s_upper = ~0ull;
    }
    __syncthreads();
    int c = 0;
    for (int j = tid; j < N; j += 256) c += !(fabs(tdb[j] - ti) < min_gap);
    atomicAdd(&s_total, c);
    __syncthreads();
    const int total = s_total;
    const int kk = min(k, total);
    const bool hf_i = gating && hfq[r] != 0;
    const int64_t fi = gating ? fq[r] : 0;
    for (int done = 0; done < kk && !s_stop; done += TOPK_LARGE) {
        const uint64_t upper = s_upper;   // keys of this window are below it (all on window 0)
        const bool first = done == 0;
        const int left = total - done;    // candidates not yet emitted
        const int want = min(kk - done, TOPK_LARGE);
        // radix select: prefix of the want-th largest key below `upper`
        uint64_t prefix = 0;
        int need = want;
        for (int d = 7; d >= 0 && want < left; --d) {
            for (int b = tid; b < 256; b += 256) hist[b] = 0;
            __syncthreads();
            const uint64_t hmask = d == 7 ? 0ull : (~0ull << (8 * (d + 1)));
            for (int j = tid; j < N; j += 256) {
                if (fabs(tdb[j] - ti) < min_gap) continue;
                const uint64_t key = knn_key(row[j], j);
                if ((!first && key >= upper) || (key & hmask) != prefix) continue;
                atomicAdd(&hist[(int)((key >> (8 * d)) & 0xff)], 1);
            }
            __syncthreads();
            if (tid == 0) {
                int acc = 0, b = 255;
                for (; b > 0; --b) {
                    if (acc + hist[b] >= need) break;
                    acc += hist[b];
                }
                s_prefix = prefix | ((uint64_t)b << (8 * d));
                s_need = need - acc;
            }
            __syncthreads();
            prefix = s_prefix;
            need = s_need;
            __syncthreads();
        }
        // gather the window's keys (every key below `upper` when the window takes the rest)
        if (tid == 0) s_n = 0;
        __syncthreads();
        for (int j = tid; j < N; j += 256) {
            if (fabs(tdb[j] - ti) < min_gap) continue;
            const uint64_t key = knn_key(row[j], j);
            if (!first && key >= upper) continue;
            if (want < left && key < prefix) continue;
            const int slot = atomicAdd(&s_n, 1);
            if (slot < TOPK_LARGE) keys[slot] = key;
        }
        __syncthreads();
        const int n = min(s_n, want);
        int P = 1;
        while (P < n) P <<= 1;
        for (int i = n + tid; i < P; i += 256) keys[i] = 0ull;  // sort to the end (descending)
        __syncthreads();
        for (int kb = 2; kb <= P; kb <<= 1)
            for (int jb = kb >> 1; jb > 0; jb >>= 1) {
                for (int i = tid; i < P; i += 256) {
                    const int ixj = i ^ jb;
                    if (ixj > i) {
                        const uint64_t a = keys[i], b = keys[ixj];
                        if (((i & kb) == 0) == (a < b)) { keys[i] = b; keys[ixj] = a; }
                    }
                }
                __syncthreads();
            }
        if (tid == 0) {
            int emitted = s_emitted, nvalid = s_nvalid;
            for (int e = 0; e < n; ++e) {
                const int j = (int)(uint32_t)keys[e];
                const float v = row[j];
                if (v < thr) {
                    s_stop = 1;
                    break;
                }
                bool ok = true;
                if (hf_i && hfdb[j]) ok = fi == fdb[j];
                idx_out[(size_t)r * k + emitted] = j;
                sim_out[(size_t)r * k + emitted] = v;
                if (valid_out) valid_out[(size_t)r * k + emitted] = ok;
                nvalid += ok;
                ++emitted;
            }
            s_emitted = emitted;
            s_nvalid = nvalid;
            if (n > 0) s_upper = keys[n - 1];
            if (n < want) s_stop = 1;
        }
        __syncthreads();
    }
    if (tid == 0) {
        count_out[r] = s_emitted;
        if (totals) {
            atomicAdd(totals + 0, (unsigned long long)s_nvalid);
            atomicAdd(totals + 1, (unsigned long long)(s_emitted - s_nvalid));
        }
    }
}

// ---------------------------------------------------------- fused path ----
// numpy pairwise-sum tree of one 8192-element chunk: leaves (<= 128 elements) in order.
// Each lane walks the same DFS; lane L sums leaves L, L + 64, ... (pairwise_leaf, the
// exact leaf order) into LDS; lane 0 then combines them in the tree's order.
__device__ float pairwise_sumsq_wave(const float* a, int n, float* leaf) {
    const int lane = threadIdx.x & 63;
    // pass 1: enumerate leaves, lane-parallel sums
    {
        int st_off[16], st_n[16], sp = 0, li = 0;
        st_off[0] = 0; st_n[0] = n;
        while (sp >= 0) {
            const int o = st_off[sp], m = st_n[sp];
            --sp;
            if (m <= 128) {
                if ((li & 63) == lane) leaf[li] = pairwise_leaf(a + o, m);
                ++li;
            } else {
                int n2 = m / 2;
                n2 -= n2 % 8;
                ++sp; st_off[sp] = o + n2; st_n[sp] = m - n2;  // right after left
                ++sp; st_off[sp] = o; st_n[sp] = n2;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    float ret = 0.f;
    if (lane == 0) {  // pass 2: post-order combine, leaves consumed in order
        int st_off[16], st_n[16], st_state[16];
        float st_val[16];
        int sp = 0, li = 0;
        st_off[0] = 0; st_n[0] = n; st_state[0] = 0;
        while (sp >= 0) {
            const int o = st_off[sp], m = st_n[sp];
            if (m <= 128) {
                ret = leaf[li++];
                --sp;
            } else {
                int n2 = m / 2;
                n2 -= n2 % 8;
                if (st_state[sp] == 0) {
                    st_state[sp] = 1;
                    ++sp; st_off[sp] = o; st_n[sp] = n2; st_state[sp] = 0;
                } else if (st_state[sp] == 1) {
                    st_val[sp] = ret;
                    st_state[sp] = 2;
                    ++sp; st_off[sp] = o + n2; st_n[sp] = m - n2; st_state[sp] = 0;
                } else {
                    ret = __fadd_rn(st_val[sp], ret);
                    --sp;
                }
            }
        }
    }
    return __shfl(ret, 0, 64);
}

__global__ __launch_bounds__(256) void k_row_norm_wave(const float* __restrict__ X, float* __restrict__ Xn, int N,
                                                       int D, float* __restrict__ norms) {
    __shared__ float leaf[4][128];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i = blockIdx.x * 4 + wave;
    if (i >= N) return;  // wave-uniform
    const float* x = X + (size_t)i * D;
    float acc = 0.f;
    for (int c0 = 0; c0 < D; c0 += 8192) {
        const float p = pairwise_sumsq_wave(x + c0, min(8192, D - c0), leaf[wave]);
        acc = c0 == 0 ? p : __fadd_rn(acc, p);
    }
    const float nrm = __fsqrt_rn(acc);
    if (norms && lane == 0) norms[i] = nrm;
    const float den = __fadd_rn(nrm, 1e-8f);
    float* y = Xn + (size_t)i * D;
    for (int j = lane; j < D; j += 64) y[j] = __fdiv_rn(x[j], den);
}

constexpr int FR = 64;    // query rows per workgroup
constexpr int FC = 128;   // database columns per tile
constexpr int FKMAX = 32;  // fused path: k <= 32 (a list rank per lane)

// Row lists in registers: lane l holds rank l of each of the wave's 16 rows.
__global__ __launch_bounds__(256, 2) void k_knn_scan(const float* __restrict__ Xq, int Q, const float* __restrict__ Xd,
                                                     int N, int D, const double* __restrict__ tq,
                                                     const double* __restrict__ tdb, double min_gap, float thr, int k,
                                                     int cols_per_split, int nsplit_arg, float* __restrict__ part_v,
                                                     int32_t* __restrict__ part_i, int32_t* __restrict__ part_n) {
    __shared__ float As[SBK][FR + 4];
    __shared__ float Bs[SBK][FC + 4];
    __shared__ float St[FR][FC + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // 1-D grid dealt XCD-major: block b runs on XCD b % 8; its local index i = b / 8 walks
    // the row blocks of one column split before the next split, so each XCD streams its
    // own splits' database rows and keeps them in its L2
    const int nrb = (Q + FR - 1) / FR, nsplit = nsplit_arg;
    const int xcd = (int)blockIdx.x & 7, i8 = (int)blockIdx.x >> 3;
    const int split = xcd + 8 * (i8 / nrb);
    if (split >= nsplit) return;
    const int r0 = (i8 % nrb) * FR;
    const int cb = split * cols_per_split, ce = min(N, cb + cols_per_split);
    if (cb >= ce) {
        for (int q = 0; q < 16; ++q) {
            const int row = r0 + wave * 16 + q;
            if (row < Q && lane == 0) part_n[(size_t)row * nsplit + split] = 0;
        }
        return;
    }
    float lv[16];
    int li[16], cnt[16];
    double ti[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        lv[q] = -INFINITY;
        li[q] = -1;
        cnt[q] = 0;
        ti[q] = tq[min(r0 + wave * 16 + q, Q - 1)];
    }
    for (int c0 = cb; c0 < ce; c0 += FC) {
        f32x16 acc[2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][r] = 0.f;
        // stage 64 rows (A) and 128 columns (B) x 16 k, transposed to [k][row]; the next
        // k-step's values are fetched into registers while this one's MFMAs run
        const float* srcs[3];
        int rows_[3], kqs[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int c = tid + i * 256, isA = c < 256;
            const int cc = isA ? c : c - 256;
            rows_[i] = cc >> 2;
            kqs[i] = (cc & 3) * 4;
            srcs[i] = isA ? Xq + (size_t)min(r0 + rows_[i], Q - 1) * D : Xd + (size_t)min(c0 + rows_[i], N - 1) * D;
        }
        auto fetch = [&](int k0, float (&tv)[3][4]) {
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int kq = kqs[i];
                if (k0 + kq + 3 < D) {
                    const float4 v = *reinterpret_cast<const float4*>(srcs[i] + k0 + kq);
                    tv[i][0] = v.x; tv[i][1] = v.y; tv[i][2] = v.z; tv[i][3] = v.w;
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) tv[i][u] = k0 + kq + u < D ? srcs[i][k0 + kq + u] : 0.f;
                }
            }
        };
        auto put = [&](const float (&tv)[3][4]) {
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (i == 0) As[kqs[i] + u][rows_[i]] = tv[i][u];
                    else Bs[kqs[i] + u][rows_[i]] = tv[i][u];
                }
        };
        float tv[3][4];
        fetch(0, tv);
        put(tv);
        __syncthreads();
        for (int k0 = 0; k0 < D; k0 += SBK) {
            const bool more = k0 + SBK < D;
            if (more) fetch(k0 + SBK, tv);
#pragma unroll
            for (int kk = 0; kk < SBK; kk += 2) {
                const int kx = kk + (lane >> 5);
                const float b = Bs[kx][wave * 32 + (lane & 31)];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
                    acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(As[kx][mt * 32 + (lane & 31)], b, acc[mt], 0, 0, 0);
            }
            __syncthreads();
            if (more) {
                put(tv);
                __syncthreads();
            }
        }
        // D[i][j]: column j = lane & 31 (of this wave's 32), row i = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                St[mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)][wave * 32 + (lane & 31)] = acc[mt][r];
        __syncthreads();
        // stream the tile into the wave's 16 row lists (lane: columns c0 + lane, c0 + 64 + lane)
        double tj[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) tj[h] = tdb[min(c0 + lane + 64 * h, N - 1)];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row = wave * 16 + q;
            const float kv = __shfl(lv[q], k - 1, 64);
            const int ki = __shfl(li[q], k - 1, 64);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = lane + 64 * h, j = c0 + c;
                const float v = St[row][c];
                bool pass = j < ce && !(fabs(tj[h] - ti[q]) < min_gap) && !(v < thr) && v > -INFINITY;
                pass = pass && (cnt[q] < k || before(v, j, kv, ki));
                unsigned long long m = __ballot(pass);
                while (m) {
                    const int src_l = __builtin_ctzll(m);
                    m &= m - 1;
                    const float cv = __shfl(v, src_l, 64);
                    const int cj = __shfl(j, src_l, 64);
                    // rank of the candidate: entries before it
                    const bool bef = lane < cnt[q] && before(lv[q], li[q], cv, cj);
                    const int pos = __popcll(__ballot(bef));
                    if (pos < k) {
                        const float up_v = __shfl_up(lv[q], 1, 64);
                        const int up_i = __shfl_up(li[q], 1, 64);
                        if (lane == pos) { lv[q] = cv; li[q] = cj; }
                        else if (lane > pos) { lv[q] = up_v; li[q] = up_i; }
                        cnt[q] = min(cnt[q] + 1, k);
                    }
                }
            }
        }
        __syncthreads();  // St is rewritten by the next tile
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int row = r0 + wave * 16 + q;
        if (row >= Q) continue;  // wave-uniform
        const size_t base = ((size_t)row * nsplit + split) * k;
        if (lane < k) {
            part_v[base + lane] = lv[q];
            part_i[base + lane] = li[q];
        }
        if (lane == 0) part_n[(size_t)row * nsplit + split] = cnt[q];
    }
}

// Merge the column splits' sorted lists of each row (one wave per row): k rounds of a
// wave argmax over the lists' heads; then the floor bit and the totals, as k_topk_gate.
__global__ __launch_bounds__(64) void k_knn_merge(const float* __restrict__ part_v, const int32_t* __restrict__ part_i,
                                                  const int32_t* __restrict__ part_n, int nsplit, int Q,
                                                  const int64_t* __restrict__ fq, const uint8_t* __restrict__ hfq,
                                                  const int64_t* __restrict__ fdb, const uint8_t* __restrict__ hfdb,
                                                  int k, int gating, int32_t* __restrict__ idx_out,
                                                  float* __restrict__ sim_out, uint8_t* __restrict__ valid_out,
                                                  int32_t* __restrict__ count_out,
                                                  unsigned long long* __restrict__ totals) {
    const int lane = threadIdx.x, r = blockIdx.x;
    if (r >= Q) return;
    // lane s < nsplit walks list s
    const bool own = lane < nsplit;
    const size_t base = ((size_t)r * nsplit + lane) * k;
    const int n = own ? part_n[(size_t)r * nsplit + lane] : 0;
    int ptr = 0;
    int emitted = 0, nvalid = 0;
    const bool hf_i = gating && hfq[r] != 0;
    const int64_t fi = gating ? fq[r] : 0;
    for (int step = 0; step < k; ++step) {
        float bv = ptr < n ? part_v[base + ptr] : -INFINITY;
        int bi = ptr < n ? part_i[base + ptr] : -1;
        const int mine = bi;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(bv, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (oi >= 0 && (bi < 0 || before(ov, oi, bv, bi))) { bv = ov; bi = oi; }
        }
        if (bi < 0) break;
        if (mine == bi) ++ptr;  // indices are distinct across splits
        if (lane == 0) {
            bool ok = true;
            if (hf_i && hfdb[bi]) ok = fi == fdb[bi];
            idx_out[(size_t)r * k + emitted] = bi;
            sim_out[(size_t)r * k + emitted] = bv;
            if (valid_out) valid_out[(size_t)r * k + emitted] = ok;
            nvalid += ok;
        }
        ++emitted;
    }
    if (lane == 0) {
        count_out[r] = emitted;
        if (totals) {
            atomicAdd(totals + 0, (unsigned long long)nvalid);
            atomicAdd(totals + 1, (unsigned long long)(emitted - nvalid));
        }
    }
}

// CricaVPR.compute_cross_correlation_score reduction: given C [n1, n2],
// score = sqrt(mean_i max_j C + ... ) -- one workgroup, fixed reduction order.
__global__ __launch_bounds__(256) void k_xcorr_reduce(const float* __restrict__ C, int n1, int n2,
                                                      float* __restrict__ out) {
    __shared__ float red[2][256];
    float rs = 0.f, cs = 0.f;
    for (int i = threadIdx.x; i < n1; i += 256) {
        float m = -INFINITY;
        for (int j = 0; j < n2; ++j) m = fmaxf(m, C[(size_t)i * n2 + j]);
        rs += m;
    }
    for (int j = threadIdx.x; j < n2; j += 256) {
        float m = -INFINITY;
        for (int i = 0; i < n1; ++i) m = fmaxf(m, C[(size_t)i * n2 + j]);
        cs += m;
    }
    red[0][threadIdx.x] = rs;
    red[1][threadIdx.x] = cs;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = sqrtf((red[0][0] / (float)n1) * (red[1][0] / (float)n2));
}

// ------------------------------------------------------- batched rerank ------
// CricaVPR.rerank_candidates at scale (place_recognition.py:714-757): the cross-
// correlation score of many (query, candidate) local-feature pairs in one pass.  Grid
// (column tile, row tile, pair): each workgroup computes one 128 x 128 tile of C = qn mn^T
// (sim_tile: the same exact-f32 MFMA k order as the single-pair mlg_xcorr_score) and keeps
// only its maxima -- every row's max over the tile's columns and every column's max over
// the tile's rows -- so no [n1, n2] matrix is written; k_xcorr_finish takes the max over
// the tiles and the means in k_xcorr_reduce's order (the same bits as the single pair).
// feats: L2-normalised rows, frame f at feats + f * L * D; rowp [P][ct][L], colp [P][rt][L].
__global__ __launch_bounds__(256, 2) void k_xcorr_tiles(const float* __restrict__ feats, int L, int D,
                                                        const int32_t* __restrict__ qa,
                                                        const int32_t* __restrict__ qb, float* __restrict__ rowp,
                                                        float* __restrict__ colp) {
    __shared__ float As[SBK][SBM + 4];
    __shared__ float Bs[SBK][SBN + 4];
    __shared__ float part[2][2][SBM];  // [row / col][wave half][index in tile]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int p = blockIdx.z, ct = blockIdx.x, rt = blockIdx.y;
    const int m0 = rt * SBM, n0 = ct * SBN;
    const int nct = gridDim.x, nrt = gridDim.y;
    const float* A = feats + (size_t)qa[p] * L * D;
    const float* B = feats + (size_t)qb[p] * L * D;
    f32x16 acc[2][2];
    sim_tile(A, L, B, L, D, m0, n0, As, Bs, acc);
    // D[i][j]: col j = lane & 31, row i = (r & 3) + 8 (r >> 2) + 4 (lane >> 5); rows / columns
    // past L are clamped copies and are masked out of both maxima
    const int hh = lane >> 5, c = lane & 31;
    float cm[2] = {-INFINITY, -INFINITY};  // column max per tb over this wave's 64 rows
#pragma unroll
    for (int ta = 0; ta < 2; ++ta)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int i = m0 + wm * 64 + ta * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            float rm = -INFINITY;
#pragma unroll
            for (int tb = 0; tb < 2; ++tb) {
                const int j = n0 + wn * 64 + tb * 32 + c;
                const float v = acc[ta][tb][r];
                if (j < L) rm = fmaxf(rm, v);
                if (i < L) cm[tb] = fmaxf(cm[tb], v);
            }
            // row max across the 32 lanes of this half (columns c)
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) rm = fmaxf(rm, __shfl_xor(rm, o, 64));
            if (c == 0) part[0][wn][wm * 64 + ta * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh] = rm;
        }
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
        const float v = fmaxf(cm[tb], __shfl_xor(cm[tb], 32, 64));  // both row halves
        if (hh == 0) part[1][wm][wn * 64 + tb * 32 + c] = v;
    }
    __syncthreads();
    if (tid < SBM) {
        const int i = m0 + tid;
        if (i < L) rowp[((size_t)p * nct + ct) * L + i] = fmaxf(part[0][0][tid], part[0][1][tid]);
    } else {
        const int j = n0 + tid - SBM;
        if (j < L) colp[((size_t)p * nrt + rt) * L + j] = fmaxf(part[1][0][tid - SBM], part[1][1][tid - SBM]);
    }
}

// one workgroup per pair: maxima over the tiles, then k_xcorr_reduce's sums and root
__global__ __launch_bounds__(256) void k_xcorr_finish(const float* __restrict__ rowp, const float* __restrict__ colp,
                                                      int L, int nct, int nrt, float* __restrict__ score) {
    __shared__ float red[2][256];
    const int p = blockIdx.x;
    float rs = 0.f, cs = 0.f;
    for (int i = threadIdx.x; i < L; i += 256) {
        float m = -INFINITY;
        for (int t = 0; t < nct; ++t) m = fmaxf(m, rowp[((size_t)p * nct + t) * L + i]);
        rs += m;
    }
    for (int j = threadIdx.x; j < L; j += 256) {
        float m = -INFINITY;
        for (int t = 0; t < nrt; ++t) m = fmaxf(m, colp[((size_t)p * nrt + t) * L + j]);
        cs += m;
    }
    red[0][threadIdx.x] = rs;
    red[1][threadIdx.x] = cs;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) score[p] = sqrtf((red[0][0] / (float)L) * (red[1][0] / (float)L));
}

}  // namespace

// pairs per k_xcorr_tiles launch: grid z stays far below the 65535 grid-dimension cap and
// the per-tile maxima (rowp / colp) take at most 2 * XC_SLICE * t * L floats of workspace
// (346 MB at L = 528) however many pairs one call scores
constexpr int XC_SLICE = 16384;

size_t mlg_xcorr_batch_ws_bytes(int F, int L, int D, int P) {
    if (F <= 0 || L <= 0 || D <= 0 || P <= 0) return 0;
    const size_t t = (size_t)((L + SBM - 1) / SBM);
    const size_t ps = (size_t)(P < XC_SLICE ? P : XC_SLICE);
    return (((size_t)F * L * D * 4 + 255) & ~(size_t)255) + 2 * ps * t * L * 4;
}

int mlg_xcorr_batch_run(const float* feats, int F, int L, int D, const int32_t* qa, const int32_t* qb, int P,
                        void* ws, size_t ws_bytes, float* score, hipStream_t s) {
    if (P <= 0) return MLG_OK;
    if (!feats || !qa || !qb || !ws || !score || F <= 0 || L <= 0 || D <= 0 || (D % 4)) return MLG_EINVAL;
    if (ws_bytes < mlg_xcorr_batch_ws_bytes(F, L, D, P)) return MLG_ENOMEM;
    float* fn = (float*)ws;
    const int t = (L + SBM - 1) / SBM;
    float* rowp = (float*)((char*)ws + (((size_t)F * L * D * 4 + 255) & ~(size_t)255));
    float* colp = rowp + (size_t)(P < XC_SLICE ? P : XC_SLICE) * t * L;
    // the reference's q / (||q|| + 1e-8) per row, numpy-exact (one thread per row)
    hipLaunchKernelGGL(k_row_normalize, dim3((F * L + 63) / 64), dim3(64), 0, s, feats, fn, F * L, D, D, nullptr);
    for (int p0 = 0; p0 < P; p0 += XC_SLICE) {  // stream order: a slice reuses rowp / colp after the last
        const int ps = P - p0 < XC_SLICE ? P - p0 : XC_SLICE;
        hipLaunchKernelGGL(k_xcorr_tiles, dim3(t, t, ps), dim3(256), 0, s, fn, L, D, qa + p0, qb + p0, rowp, colp);
        hipLaunchKernelGGL(k_xcorr_finish, dim3(ps), dim3(256), 0, s, rowp, colp, L, t, t, score + p0);
    }
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_row_normalize(const float* X, float* Xn, int N, int D, float* norms, hipStream_t s) {
    if (N <= 0 || D <= 0) return MLG_EINVAL;
    hipLaunchKernelGGL(k_row_normalize, dim3((N + 63) / 64), dim3(64), 0, s, X, Xn, N, D, D, norms);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_similarity_f32(const float* A, int Q, const float* B, int N, int D, float* S, int lds, hipStream_t s) {
    return mlg_similarity_f32_t(A, Q, B, N, D, S, lds, nullptr, 0, s);
}

int mlg_similarity_f32_t(const float* A, int Q, const float* B, int N, int D, float* S, int lds, float* St, int ldt,
                         hipStream_t s) {
    if (N <= 0 || D <= 0 || Q <= 0 || (D % 4) || lds < N) return MLG_EINVAL;
    if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return MLG_EINVAL;
    if (St && (ldt < Q || (ldt % 4) || (reinterpret_cast<uintptr_t>(St) & 15))) return MLG_EINVAL;
    dim3 grid((N + SBN - 1) / SBN, (Q + SBM - 1) / SBM);
    hipLaunchKernelGGL(k_sim_f32<false>, grid, dim3(256), 0, s, A, Q, B, N, D, S, lds, St, ldt);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_similarity_f32_loftr(const float* A, int Q, const float* B, int N, int D, float* S, int lds, hipStream_t s) {
    if (N <= 0 || D <= 0 || Q <= 0 || (D % 4) || lds < N) return MLG_EINVAL;
    if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return MLG_EINVAL;
    dim3 grid((N + SBN - 1) / SBN, (Q + SBM - 1) / SBM);
    hipLaunchKernelGGL(k_sim_f32<true>, grid, dim3(256), 0, s, A, Q, B, N, D, S, lds, (float*)nullptr, 0);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_topk_gate(const float* S, int lds, int N, int Q, const double* tq, const double* tdb, const int64_t* fq,
                  const uint8_t* hfq, const int64_t* fdb, const uint8_t* hfdb, double min_gap, float thr, int k,
                  int gating, int32_t* idx, float* sim, uint8_t* valid, int32_t* count, unsigned long long* totals,
                  hipStream_t s) {
    if (N <= 0 || Q <= 0 || k <= 0 || lds < N) return MLG_EINVAL;
    if (gating && (!fq || !hfq || !fdb || !hfdb)) return MLG_EINVAL;
    if (k > 256)
        hipLaunchKernelGGL(k_topk_large, dim3(Q), dim3(256), 0, s, S, lds, N, Q, tq, tdb, fq, hfq, fdb, hfdb, min_gap,
                           thr, k, gating, idx, sim, valid, count, totals);
    else if (k <= 32)
        hipLaunchKernelGGL(k_topk_gate<32>, dim3(Q), dim3(64), 0, s, S, lds, N, Q, tq, tdb, fq, hfq, fdb, hfdb,
                           min_gap, thr, k, gating, idx, sim, valid, count, totals);
    else
        hipLaunchKernelGGL(k_topk_gate<256>, dim3(Q), dim3(64), 0, s, S, lds, N, Q, tq, tdb, fq, hfq, fdb, hfdb,
                           min_gap, thr, k, gating, idx, sim, valid, count, totals);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_xcorr_reduce(const float* C, int n1, int n2, float* out, hipStream_t s) {
    if (n1 <= 0 || n2 <= 0) return MLG_EINVAL;
    hipLaunchKernelGGL(k_xcorr_reduce, dim3(1), dim3(256), 0, s, C, n1, n2, out);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_row_normalize_wave(const float* X, float* Xn, int N, int D, float* norms, hipStream_t s) {
    if (N <= 0 || D <= 0) return MLG_EINVAL;
    hipLaunchKernelGGL(k_row_norm_wave, dim3((N + 3) / 4), dim3(256), 0, s, X, Xn, N, D, norms);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

size_t mlg_knn_fused_ws_bytes(int Q, int N, int k) {
    const int nsplit = mlg_knn_fused_splits(Q, N);
    return (size_t)Q * nsplit * ((size_t)k * 8 + 4) + 256;
}

int mlg_knn_fused_splits(int Q, int N) {
    // a multiple of the 8 XCDs; each split's database rows (<= ~2 MB) fit an XCD's 4 MB
    // L2; at least 512 workgroups (256 CUs x 2) when the rows allow
    const int rb = (Q + FR - 1) / FR;
    const long split_bytes_cap = 2L << 20;
    int ns = 8;
    while (ns < 64 && ((long)N * 768 * 4 / ns > split_bytes_cap || (long)rb * ns < 512)) ns += 8;
    return ns;
}

int mlg_knn_fused(const float* Xq, int Q, const float* Xd, int N, int D, const double* tq, const double* tdb,
                  const int64_t* fq, const uint8_t* hfq, const int64_t* fdb, const uint8_t* hfdb, double min_gap,
                  float thr, int k, int gating, void* ws, int32_t* idx, float* sim, uint8_t* valid, int32_t* count,
                  unsigned long long* totals, hipStream_t s) {
    if (Q <= 0 || N <= 0 || D <= 0 || (D % 4) || k <= 0 || k > FKMAX) return MLG_EINVAL;
    if (gating && (!fq || !hfq || !fdb || !hfdb)) return MLG_EINVAL;
    const int nsplit = mlg_knn_fused_splits(Q, N);
    const int tiles = (N + FC - 1) / FC;
    const int cps = ((tiles + nsplit - 1) / nsplit) * FC;
    float* pv = (float*)ws;
    int32_t* pi = (int32_t*)(pv + (size_t)Q * nsplit * k);
    int32_t* pn = pi + (size_t)Q * nsplit * k;
    const int nrb = (Q + FR - 1) / FR;
    const int grid = 8 * nrb * ((nsplit + 7) / 8);
    hipLaunchKernelGGL(k_knn_scan, dim3(grid), dim3(256), 0, s, Xq, Q, Xd, N, D, tq, tdb, min_gap, thr, k, cps, nsplit,
                       pv, pi, pn);
    MLG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_knn_merge, dim3(Q), dim3(64), 0, s, pv, pi, pn, nsplit, Q, fq, hfq, fdb, hfdb, k, gating, idx,
                       sim, valid, count, totals);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}
