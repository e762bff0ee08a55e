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

__global__ __launch_bounds__(256, 2) void k_sim_f32(const float* __restrict__ A, int Q, const float* __restrict__ B,
                                                    int N, int D, float* __restrict__ S, int lds) {
    __shared__ float As[SBK][SBM + 4];
    __shared__ float Bs[SBK][SBN + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m0 = blockIdx.y * SBM, n0 = blockIdx.x * SBN;
    const int wm = wave >> 1, wn = wave & 1;
    f32x16 acc[2][2];
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

}  // namespace

int mlg_row_normalize(const float* X, float* Xn, int N, int D, float* norms, hipStream_t s) {
    if (N <= 0 || D <= 0) return MLG_EINVAL;
    hipLaunchKernelGGL(k_row_normalize, dim3((N + 63) / 64), dim3(64), 0, s, X, Xn, N, D, D, norms);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_similarity_f32(const float* A, int Q, const float* B, int N, int D, float* S, int lds, hipStream_t s) {
    if (N <= 0 || D <= 0 || Q <= 0 || (D % 4) || lds < N) return MLG_EINVAL;
    if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return MLG_EINVAL;
    dim3 grid((N + SBN - 1) / SBN, (Q + SBM - 1) / SBM);
    hipLaunchKernelGGL(k_sim_f32, grid, dim3(256), 0, s, A, Q, B, N, D, S, lds);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_topk_gate(const float* S, int lds, int N, int Q, const double* tq, const double* tdb, const int64_t* fq,
                  const uint8_t* hfq, const int64_t* fdb, const uint8_t* hfdb, double min_gap, float thr, int k,
                  int gating, int32_t* idx, float* sim, uint8_t* valid, int32_t* count, unsigned long long* totals,
                  hipStream_t s) {
    if (N <= 0 || Q <= 0 || k <= 0 || k > 256 || lds < N) return MLG_EINVAL;
    if (gating && (!fq || !hfq || !fdb || !hfdb)) return MLG_EINVAL;
    if (k <= 32)
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
