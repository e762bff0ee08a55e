// Trajectory-proximity loop-closure candidates + fused floor gate.
//
// Restates detect_loop_closure_candidates + apply_floor_gating of the SLAM
// integrations (orb_slam3_integration.py:167-281, lego_loam_integration.py:121-204):
//   every pair (i, j) with j - i >= min_gap and ||p_i - p_j|| <= r, emitted in (i, j)
//   order with dist = ||p_i - p_j|| and the strict / non-strict floor verdict of
//   SemanticLoopClosureGate.gate_candidate (loop_closure_gate.py:60-99).
// The inclusion test is the one scipy's KD-tree applies for p = 2: the float64 sum
// ((dx*dx + dy*dy) + dz*dz), uncontracted, compared with r*r.
//
// Two passes over (row block x j-chunk) tiles; the pair set is never materialised
// densely.  Pass 1 counts, per (row, chunk), total and accepted pairs packed into
// one uint64 (total | accepted << 32); an exclusive scan of that array (rocPRIM)
// gives each (row, chunk) its output offset in (i, j) order; pass 2 recomputes the
// tile and writes.  Positions of one j-chunk are staged in LDS as SoA doubles so
// the inner loop is a wave-uniform broadcast read.
#include <rocprim/device/device_scan.hpp>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int PX_ROWS = 256;  // rows (threads) per workgroup
constexpr int PX_JC = 2048;   // j positions per chunk (48 KB of LDS)

#pragma clang fp contract(off)
__device__ __forceinline__ double sqdist(double ax, double ay, double az, double bx, double by, double bz) {
    const double dx = ax - bx, dy = ay - by, dz = az - bz;
    return (dx * dx + dy * dy) + dz * dz;
}

template <bool EMIT>
__global__ __launch_bounds__(PX_ROWS) void k_proximity(const double* __restrict__ pos, const int64_t* __restrict__ floor,
                                                       int N, int row0, int nrows, double r2, int min_gap,
                                                       int floor_limit, int nchunk, uint64_t* __restrict__ counts,
                                                       const uint64_t* __restrict__ offsets, int32_t* __restrict__ pairs,
                                                       double* __restrict__ dist, uint8_t* __restrict__ valid) {
    __shared__ double sx[PX_JC], sy[PX_JC], sz[PX_JC];
    __shared__ int64_t sf[PX_JC];
    const int c = blockIdx.y;
    const int jbeg = c * PX_JC, jend = min(N, jbeg + PX_JC);
    const int rb0 = row0 + blockIdx.x * PX_ROWS;  // first row of this block
    // Skip tiles entirely below the diagonal band (every j < i + min_gap).
    if (jend - 1 < rb0 + min_gap) {
        if (!EMIT) {
            const int rl = blockIdx.x * PX_ROWS + threadIdx.x;
            if (rl < nrows) counts[(size_t)rl * nchunk + c] = 0;
        }
        return;
    }
    for (int k = threadIdx.x; k < jend - jbeg; k += PX_ROWS) {
        const double* p = pos + (size_t)(jbeg + k) * 3;
        sx[k] = p[0];
        sy[k] = p[1];
        sz[k] = p[2];
        sf[k] = floor ? floor[jbeg + k] : 0;
    }
    __syncthreads();
    const int rl = blockIdx.x * PX_ROWS + threadIdx.x;
    const int i = row0 + rl;
    const bool live = rl < nrows;
    const double px = live ? pos[(size_t)i * 3 + 0] : 0.0;
    const double py = live ? pos[(size_t)i * 3 + 1] : 0.0;
    const double pz = live ? pos[(size_t)i * 3 + 2] : 0.0;
    const int64_t fi = (live && floor) ? floor[i] : 0;
    const int jlo = live ? max(jbeg, i + min_gap) : jend;
    // wave-uniform loop start: the smallest jlo of the wave (lanes below their own jlo idle)
    int wlo = jlo;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wlo = min(wlo, __shfl_xor(wlo, o, 64));
    uint32_t tot = 0, acc = 0;
    size_t out = 0;
    if (EMIT && live) {
        const uint64_t o = offsets[(size_t)rl * nchunk + c];
        out = (uint32_t)o;
    }
    for (int j = wlo; j < jend; ++j) {
        const int k = j - jbeg;
        const double d2 = sqdist(px, py, pz, sx[k], sy[k], sz[k]);
        if (j >= jlo && d2 <= r2) {
            const int64_t df = fi - sf[k];
            const bool ok = (df < 0 ? -df : df) <= floor_limit;
            if (EMIT) {
                pairs[2 * out] = i;
                pairs[2 * out + 1] = j;
                dist[out] = sqrt(d2);
                valid[out] = ok;
                ++out;
            } else {
                ++tot;
                acc += ok;
            }
        }
    }
    if (!EMIT && live) counts[(size_t)rl * nchunk + c] = (uint64_t)tot | ((uint64_t)acc << 32);
}

__global__ void k_proximity_totals(const uint64_t* counts, const uint64_t* offsets, size_t M, long long* totals) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const uint64_t s = M ? offsets[M - 1] + counts[M - 1] : 0;
        totals[0] = (long long)(uint32_t)s;
        totals[1] = (long long)(s >> 32);
    }
}

struct ProxLayout {
    int nchunk;
    size_t M, counts, offsets, scan_tmp, scan_bytes, total;
};

ProxLayout prox_layout(int N, int nrows) {
    ProxLayout L;
    L.nchunk = (N + PX_JC - 1) / PX_JC;
    L.M = (size_t)nrows * L.nchunk;
    size_t scan_bytes = 0;
    (void)rocprim::exclusive_scan(nullptr, scan_bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, L.M,
                            rocprim::plus<uint64_t>(), (hipStream_t)0);
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    L.counts = 0;
    L.offsets = up(L.M * 8);
    L.scan_tmp = L.offsets + up(L.M * 8);
    L.scan_bytes = scan_bytes;
    L.total = L.scan_tmp + up(scan_bytes > 0 ? scan_bytes : 1);
    return L;
}

}  // namespace

// pairs per pass are bounded by 2^32 - 1 (packed counters): N <= 65536.
bool mlg_proximity_shape_ok(int N, int row0, int nrows) {
    return N >= 0 && N <= 65536 && row0 >= 0 && nrows >= 0 && row0 + nrows <= N;
}

size_t mlg_proximity_ws_bytes(int N, int nrows) {
    if (!mlg_proximity_shape_ok(N, 0, nrows)) return 0;
    return prox_layout(N, nrows).total;
}

int mlg_proximity_count_run(const double* pos, const int64_t* floor, int N, int row0, int nrows, double radius,
                            int min_gap, int strict, void* ws, size_t ws_bytes, long long* totals, hipStream_t s) {
    if (!mlg_proximity_shape_ok(N, row0, nrows) || min_gap < 1 || !(radius >= 0.0)) return MLG_EINVAL;
    const ProxLayout L = prox_layout(N, nrows);
    if (ws_bytes < L.total) return MLG_EINVAL;
    char* w = (char*)ws;
    uint64_t* counts = (uint64_t*)(w + L.counts);
    uint64_t* offsets = (uint64_t*)(w + L.offsets);
    if (L.M > 0) {
        dim3 grid((nrows + PX_ROWS - 1) / PX_ROWS, L.nchunk);
        hipLaunchKernelGGL(k_proximity<false>, grid, dim3(PX_ROWS), 0, s, pos, floor, N, row0, nrows, radius * radius,
                           min_gap, strict ? 0 : 1, L.nchunk, counts, nullptr, nullptr, nullptr, nullptr);
        MLG_LAUNCH_CHECK();
        size_t sb = L.scan_bytes;
        if (rocprim::exclusive_scan(w + L.scan_tmp, sb, counts, offsets, (uint64_t)0, L.M, rocprim::plus<uint64_t>(),
                                    s) != hipSuccess)
            return MLG_EHIP;
    }
    hipLaunchKernelGGL(k_proximity_totals, dim3(1), dim3(64), 0, s, counts, offsets, L.M, totals);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

int mlg_proximity_emit_run(const double* pos, const int64_t* floor, int N, int row0, int nrows, double radius,
                           int min_gap, int strict, const void* ws, size_t ws_bytes, int32_t* pairs, double* dist,
                           uint8_t* valid, hipStream_t s) {
    if (!mlg_proximity_shape_ok(N, row0, nrows) || min_gap < 1 || !(radius >= 0.0)) return MLG_EINVAL;
    const ProxLayout L = prox_layout(N, nrows);
    if (ws_bytes < L.total) return MLG_EINVAL;
    if (L.M == 0) return MLG_OK;
    const char* w = (const char*)ws;
    dim3 grid((nrows + PX_ROWS - 1) / PX_ROWS, L.nchunk);
    hipLaunchKernelGGL(k_proximity<true>, grid, dim3(PX_ROWS), 0, s, pos, floor, N, row0, nrows, radius * radius,
                       min_gap, strict ? 0 : 1, L.nchunk, nullptr, (const uint64_t*)(w + L.offsets), pairs, dist,
                       valid);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}
