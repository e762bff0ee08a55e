// Batched ground-plane RANSAC for the LiDAR floor tracker
// (lidar_floor_tracker.py:92-141, LiDARFloorTracker.fit_ground_plane_ransac).
//
// Per scan: `iterations` hypotheses, each 3 distinct random ground points -> unit
// normal n = (p2 - p1) x (p3 - p1) / |.| (skipped when |.| < 1e-6), d = -n . p1;
// inliers = #(|P n + d| < threshold) in float64, best = most inliers (first hypothesis
// on ties, as the reference's strict `>`), ratio = best / n_points.  The reference
// draws its samples from numpy's global RNG (unseeded); here hypothesis h of a scan
// uses a counter-based stream of (seed, h), so results are deterministic and do not
// depend on the batch.  One workgroup per (scan, 64 hypotheses); the scan's points
// stream through LDS in chunks and are read by all hypotheses (broadcast).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int PL_CHUNK = 2048;  // points per LDS stage (3 floats each)

__device__ __forceinline__ uint64_t pl_mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(64) void k_plane_score(const float* __restrict__ pts, const int32_t* __restrict__ offs,
                                                    int H, uint64_t seed, double thr, double* __restrict__ planes,
                                                    int32_t* __restrict__ counts) {
    __shared__ float sp[PL_CHUNK * 3];
    const int sc = blockIdx.y;
    const int h = blockIdx.x * 64 + threadIdx.x;
    const int p0 = offs[sc], n = offs[sc + 1] - offs[sc];
    const float* P = pts + (size_t)p0 * 3;
    bool ok = h < H && n >= 3;
    double nx = 0, ny = 0, nz = 0, d = 0;
    if (ok) {
        uint64_t st = pl_mix(seed ^ (uint64_t)h * 0x632BE59BD9B4E019ull);
        int idx[3];
        for (int i = 0; i < 3; ++i) {
            int v;
            bool dup;
            do {
                st = pl_mix(st);
                v = (int)((st >> 11) % (uint64_t)n);
                dup = false;
                for (int j = 0; j < i; ++j) dup |= idx[j] == v;
            } while (dup);
            idx[i] = v;
        }
        const double ax = P[3 * idx[0]], ay = P[3 * idx[0] + 1], az = P[3 * idx[0] + 2];
        const double v1x = P[3 * idx[1]] - ax, v1y = P[3 * idx[1] + 1] - ay, v1z = P[3 * idx[1] + 2] - az;
        const double v2x = P[3 * idx[2]] - ax, v2y = P[3 * idx[2] + 1] - ay, v2z = P[3 * idx[2] + 2] - az;
        nx = v1y * v2z - v1z * v2y;
        ny = v1z * v2x - v1x * v2z;
        nz = v1x * v2y - v1y * v2x;
        const double len = sqrt(nx * nx + ny * ny + nz * nz);
        if (len < 1e-6) {
            ok = false;
        } else {
            nx /= len;
            ny /= len;
            nz /= len;
            d = -(nx * ax + ny * ay + nz * az);
        }
    }
    int cnt = 0;
    for (int c0 = 0; c0 < n; c0 += PL_CHUNK) {
        const int cn = min(PL_CHUNK, n - c0);
        __syncthreads();
        for (int i = threadIdx.x; i < cn * 3; i += 64) sp[i] = P[(size_t)c0 * 3 + i];
        __syncthreads();
        if (ok)
            for (int i = 0; i < cn; ++i) {
                const double dist = fabs(((double)sp[3 * i] * nx + (double)sp[3 * i + 1] * ny) +
                                         (double)sp[3 * i + 2] * nz + d);
                cnt += dist < thr;
            }
    }
    if (h < H) {
        counts[(size_t)sc * H + h] = ok ? cnt : -1;
        double* pl = planes + ((size_t)sc * H + h) * 4;
        pl[0] = nx;
        pl[1] = ny;
        pl[2] = nz;
        pl[3] = d;
    }
}

// per scan: the first hypothesis with the most inliers (strictly more than the best so
// far, starting from 0 as the reference does) -> plane [4] (NaN when none), ratio
__global__ void k_plane_select(const int32_t* __restrict__ offs, int H, const double* __restrict__ planes,
                               const int32_t* __restrict__ counts, double* __restrict__ best_plane,
                               double* __restrict__ ratio, int32_t* __restrict__ best_count) {
    const int sc = blockIdx.x;
    __shared__ int bc[256], bi[256];
    int c = 0, i0 = 0x7fffffff;
    for (int h = threadIdx.x; h < H; h += 256) {
        const int v = counts[(size_t)sc * H + h];
        if (v > c || (v == c && v > 0 && h < i0)) { c = v; i0 = h; }
    }
    bc[threadIdx.x] = c;
    bi[threadIdx.x] = i0;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            const int v = bc[threadIdx.x + o], j = bi[threadIdx.x + o];
            if (v > bc[threadIdx.x] || (v == bc[threadIdx.x] && j < bi[threadIdx.x])) {
                bc[threadIdx.x] = v;
                bi[threadIdx.x] = j;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int n = offs[sc + 1] - offs[sc];
        const bool have = bc[0] > 0;
        for (int k = 0; k < 4; ++k) best_plane[sc * 4 + k] = have ? planes[((size_t)sc * H + bi[0]) * 4 + k] : NAN;
        ratio[sc] = n > 0 ? (double)bc[0] / n : 0.0;
        best_count[sc] = bc[0];
    }
}

}  // namespace

size_t mlg_plane_ws_bytes(int S, int H) {
    if (S <= 0 || H <= 0) return 0;
    return (((size_t)S * H * 4 * 8 + 255) & ~(size_t)255) + (size_t)S * H * 4;
}

int mlg_plane_ransac_run(const float* pts, const int32_t* offs, int S, int H, uint64_t seed, double thr, void* ws,
                         size_t ws_bytes, double* plane, double* ratio, int32_t* inliers, hipStream_t s) {
    if (S <= 0 || H <= 0 || !(thr > 0.0)) return MLG_EINVAL;
    if (ws_bytes < mlg_plane_ws_bytes(S, H)) return MLG_EINVAL;
    double* planes = (double*)ws;
    int32_t* counts = (int32_t*)((char*)ws + (((size_t)S * H * 4 * 8 + 255) & ~(size_t)255));
    hipLaunchKernelGGL(k_plane_score, dim3((H + 63) / 64, S), dim3(64), 0, s, pts, offs, H, seed, thr, planes, counts);
    MLG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_plane_select, dim3(S), dim3(256), 0, s, offs, H, planes, counts, plane, ratio, inliers);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}
