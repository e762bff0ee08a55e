// LightGlue block projections (upstream SelfBlock.Wqkv + rotary encoding, CrossBlock
// to_qk / to_v; LightGlue(features='superpoint') as called by
// LightGlue._detect_and_match_native, scripts/semantic_gating/geometric_verification.py:
// 263-312) over the flat token layout, writing the attention operands directly:
//   Q, K  bf16 [4 heads][Npad][64]                 (self: q, k rotated; cross: qk)
//   V^T   bf16 [4][Npad / 64][64 d][64 keys]       (attention.hip's tiled V^T)
// Rows outside live segments are written as zeros.
//
// One workgroup = 8 waves = 64 tokens x one 256-column part (q, k or v) of the
// projection; the bf16 x tile [64][256] sits in LDS (XOR-swizzled 16-B chunks), the
// weights stream from L2, packed k-step-major [16][N][16] so each wave-instruction
// reads one contiguous 1 KiB, in a 4-step register ring.  Wave w owns output columns
// 32 w .. +32 of the part for both 32-token m-tiles.  The q / k parts compute
// C^T = W . X^T, which hands a lane 4 consecutive head dims of one token (the rotary
// pairs are lane-local, one 8-B store per lane); the v part swaps the MFMA operands,
// C = X . W^T, which hands a lane 4 consecutive tokens of one dim: one 8-B store into
// the transposed V^T row, where the transposed product would need 4 scattered 2-B
// stores.  Same fragments, operand order only.
#include <stdlib.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"

// Build-time A/B knobs (separate builds loaded through tools/ab_run.py; the defaults are
// the product): tile height, persistent weights-resident form, timing probes.
#ifndef MLG_PROJ_MT
#define MLG_PROJ_MT 2
#endif
#ifndef MLG_PROJ_RES
#define MLG_PROJ_RES 1
#endif
#ifndef MLG_PROJ_PROBE
#define MLG_PROJ_PROBE 0
#endif
#ifndef MLG_PROJ_PIPE
#define MLG_PROJ_PIPE 1  // the resident form with the epilogue inside the next tile's GEMM
#endif
#ifndef MLG_PROJ_SWAP
#define MLG_PROJ_SWAP 1  // pipelined form: whole 16-B staging chunks (permlane32 swap), b128 writes
#endif

namespace {

constexpr int ROWB = 512;  // LDS bytes per token row: 256 bf16

// chunk c (0..31) of row r at slot c ^ (r & 15): the 16 lanes of a ds_read_b128 lane
// group (rows {0-3,12-15,20-27} + 32 k, one chunk) hit 16 distinct bank quads.
__device__ __forceinline__ int xoff(int row, int chunk) { return row * ROWB + ((chunk ^ (row & 15)) << 4); }

__device__ __forceinline__ bf16x8 ld16(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// a tile's rotary factors: 16 KiB, [16 pairs][64 rows] float4 (common.h lg_fac4); a lane
// reads the float4 of its row for one frequency pair: the 32 lanes of a half-wave read 512
// contiguous bytes, one conflict-free ds_read_b128 (the [64][32] cos / sin images before
// round 5 took two ds_read_b64 with 2-way conflicts, profiles/r05c_lds_conflict_calibration.txt)
__device__ __forceinline__ float4 fac_tile(const float* fc, int r, int p) {
    return *reinterpret_cast<const float4*>(fc + ((p * 64 + r) << 2));
}

// Output staging image over the dead x tile: [4 heads][64 rows][64] bf16, 16-B chunk c of
// row r at slot c ^ (r & 7).  Rows are tokens for q / k and head dims for V^T; either way
// a head's 64 rows are ONE contiguous 8 KiB block of the destination, written as whole
// 1 KiB pieces (per-lane 8-B stores at a 128-B row stride touched 32 lines each).
// (A swizzle on r >> 1, 2-way instead of 4-way bank conflicts on the epilogue's writes,
// measured no faster.  The pipelined form, the product, stages through stage_pair_off
// instead: whole 16-B chunks, b128 writes, profiles/r05u_ab_proj_staging.txt.)
template <int R>
__device__ __forceinline__ int stage_off(int h, int row, int e) {
    return (h * R + row) * 128 + ((((e >> 3) ^ (row & 7))) << 4) + (e & 7) * 2;
}

// acc[mt] over K = 256 (16 k-steps; step ks: LDS chunk 2 ks + hh, W slab ks).
// SWAP: acc = X . W^T (lane col = output column), else acc = W . X^T (lane col = token).
template <bool SWAP, int MT>
__device__ __forceinline__ void proj_gemm(const bf16_t* __restrict__ wrow, size_t step, const char* lds,
                                          f32x16 (&acc)[MT]) {
    const int lane = threadIdx.x & 63, col = lane & 31, hh = lane >> 5;
    const char* xrow = lds + col * ROWB;
    const int sw = col & 15;
    bf16x8 wf[4], xa[MT], xb[MT];
#pragma unroll
    for (int s = 0; s < 4; ++s) wf[s] = ld16(wrow + s * step);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) xa[mt] = *reinterpret_cast<const bf16x8*>(xrow + 32 * mt * ROWB + ((hh ^ sw) << 4));
#pragma unroll 1
    for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int ks = 4 * kb + s;
            const int cn = ((2 * min(ks + 1, 15) + hh) ^ sw) << 4;
            bf16x8(&cur)[MT] = (s & 1) ? xb : xa;
            bf16x8(&nxt)[MT] = (s & 1) ? xa : xb;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) nxt[mt] = *reinterpret_cast<const bf16x8*>(xrow + 32 * mt * ROWB + cn);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
                acc[mt] = SWAP ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[mt], wf[s], acc[mt], 0, 0, 0)
                               : __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s], cur[mt], acc[mt], 0, 0, 0);
            wf[s] = ld16(wrow + min(ks + 4, 15) * step);
            __builtin_amdgcn_sched_barrier(0);  // keep the refill here (lg_ffn.hip)
        }
    }
}

// Bias (+ rotary), live-row mask, staging through the dead x tile `lds` and the
// coalesced copy-out of one R-token tile of part `part` (the caller has barriered after
// the GEMM's last LDS read).
// FAC_LDS (resident form): the tile's rotary factors sit in LDS at `efac` (its 16 KiB
// lg_fac4 block) instead of the global table, `bias` is this part's 256
// biases in LDS and `live` the tile's R live bytes in LDS (no global load in the epilogue).
template <bool SELF, int MT, bool FAC_LDS = false>
__device__ __forceinline__ void proj_epilogue(const f32x16 (&acc)[MT], bool is_v, int part, int m0, int nrow_,
                                              char* lds, const float* __restrict__ bias,
                                              const float* __restrict__ efac, const uint8_t* __restrict__ live,
                                              bf16_t* __restrict__ Q, bf16_t* __restrict__ K, bf16_t* __restrict__ Vt,
                                              int Npad) {
    constexpr int R = 32 * MT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 31, hh = lane >> 5;
    const int nrow = nrow_ & 0xffff;  // bit 16: timing probe, no copy-out
    if (!is_v) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = 32 * wave + 8 * g + 4 * hh;  // column within the part
            const int h = n >> 6, d = n & 63;
            const float4 b = *reinterpret_cast<const float4*>(bias + (FAC_LDS ? 0 : 256 * part) + n);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const int r = 32 * mt + col, m = min(m0 + r, Npad - 1);  // rows >= Npad: never stored
                const f32x16& a = acc[mt];
                float x0 = a[4 * g] + b.x, x1 = a[4 * g + 1] + b.y, x2 = a[4 * g + 2] + b.z, x3 = a[4 * g + 3] + b.w;
                if (SELF) {  // t * cos + rotate_half(t) * sin, uncontracted as torch
                    // (cos, sin) of frequencies d/2, d/2 + 1 (one lg_fac4 float4), read after
                    // the GEMM (held across it they cost 32 VGPRs = one workgroup per CU
                    // less): from the tile's LDS block (resident form) or global
                    const int p = (n & 63) >> 2;
                    const float4 cs = FAC_LDS ? fac_tile(efac, r, p)
                                              : reinterpret_cast<const float4*>(efac)[lg_fac4((size_t)m, p)];
                    const float2 e0 = make_float2(cs.x, cs.z), e1 = make_float2(cs.y, cs.w);
                    const float r0 = __fadd_rn(__fmul_rn(x0, e0.x), __fmul_rn(-x1, e0.y));
                    const float r1 = __fadd_rn(__fmul_rn(x1, e0.x), __fmul_rn(x0, e0.y));
                    const float r2 = __fadd_rn(__fmul_rn(x2, e1.x), __fmul_rn(-x3, e1.y));
                    const float r3 = __fadd_rn(__fmul_rn(x3, e1.x), __fmul_rn(x2, e1.y));
                    x0 = r0; x1 = r1; x2 = r2; x3 = r3;
                }
                uint2 o = make_uint2(0u, 0u);
                if (live[FAC_LDS ? r : m]) o = make_uint2(pack_bf16x2(x0, x1), pack_bf16x2(x2, x3));
                *reinterpret_cast<uint2*>(lds + stage_off<R>(h, r, d)) = o;
            }
        }
    } else {
        const int n = 32 * wave + col, h = n >> 6, d = n & 63;
        const float b = bias[(FAC_LDS ? 0 : 256 * part) + n];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const int r = 32 * mt + 8 * g + 4 * hh, m = m0 + r;  // 4 consecutive tokens
                const f32x16& a = acc[mt];
                const uint32_t lv = r < nrow ? *reinterpret_cast<const uint32_t*>(live + (FAC_LDS ? r : m)) : 0u;
                const float v0 = (lv & 0xff) ? a[4 * g] + b : 0.f;
                const float v1 = (lv & 0xff00) ? a[4 * g + 1] + b : 0.f;
                const float v2 = (lv & 0xff0000) ? a[4 * g + 2] + b : 0.f;
                const float v3 = (lv >> 24) ? a[4 * g + 3] + b : 0.f;
                // V^T staging rows: (64-key block of the tile) * 64 + d
                *reinterpret_cast<uint2*>(lds + stage_off<R>(h, (r >> 6) * 64 + d, r & 63)) =
                    make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
            }
    }
    __syncthreads();
    // copy-out: per head one contiguous [R rows][64] block at (h * Npad + m0) * 64 (for
    // V^T the R / 64 tiled [64 d][64 keys] blocks of the tile's keys, also contiguous)
    bf16_t* dst = is_v ? Vt : (part == 0 ? Q : K);
#pragma unroll
    for (int p = 0; p < R / 16; ++p) {
        const int L = p * 512 + tid, h = L / (8 * R), row = (L >> 3) % R, c = L & 7;
        if (row < nrow && !(nrow_ >> 16))
            *reinterpret_cast<uint4*>(dst + ((size_t)h * Npad + m0 + row) * 64 + c * 8) =
                *reinterpret_cast<const uint4*>(lds + stage_off<R>(h, row, 8 * c));
    }
}

// MT 32-token m-tiles per workgroup (R = 32 MT tokens; default 2, see mlg_lg_proj).
template <bool SELF, int MT>
__global__ __launch_bounds__(512) void k_lg_proj(const bf16_t* __restrict__ xcopy, int ldx,
                                                const bf16_t* __restrict__ W, const float* __restrict__ bias,
                                                const float* __restrict__ efac, const uint8_t* __restrict__ live,
                                                bf16_t* __restrict__ Q, bf16_t* __restrict__ K, bf16_t* __restrict__ Vt,
                                                int Npad) {
    constexpr int N = SELF ? 768 : 512;
    constexpr int R = 32 * MT;
    __shared__ __attribute__((aligned(16))) char lds[R * ROWB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 31, hh = lane >> 5;
    // 1-D grid, dealt so the parts (q, k, v / qk, v) of one token tile are consecutive
    // workgroups of one XCD (hardware deals block b to XCD b % 8): the tile's x rows are
    // then read from HBM once and from that XCD's L2 by the other parts (with the part in
    // blockIdx.y every part re-read the whole of x from HBM)
    constexpr int NPART = SELF ? 3 : 2;
    const int per_xcd = (int)gridDim.x >> 3;
    const int logical = ((int)blockIdx.x & 7) * per_xcd + ((int)blockIdx.x >> 3);
    if (logical >= ((Npad + R - 1) / R) * NPART) return;
    const int m0 = (logical / NPART) * R, part = logical % NPART;
    const bool is_v = part == (SELF ? 2 : 1);
    const int nrow = min(R, Npad - m0);  // a multiple of 64
#pragma unroll
    for (int i = 0; i < R / 16; ++i) {
        const int f = i * 512 + tid, row = f >> 5, c = f & 31;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (row < nrow) v = *reinterpret_cast<const uint4*>(xcopy + (size_t)(m0 + row) * ldx + c * 8);
        *reinterpret_cast<uint4*>(lds + xoff(row, c)) = v;
    }
    __syncthreads();

    const int nb = 256 * part + 32 * wave;  // first output column (row of W) of this wave
    const bf16_t* wrow = W + (size_t)(nb + col) * 16 + 8 * hh;
    f32x16 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[mt][i] = 0.f;

    if (!is_v) {
        proj_gemm<false, MT>(wrow, (size_t)N * 16, lds, acc);
    } else {
        proj_gemm<true, MT>(wrow, (size_t)N * 16, lds, acc);
    }
    __syncthreads();  // every wave has read the x tile
    proj_epilogue<SELF, MT>(acc, is_v, part, m0, nrow, lds, bias, efac, live, Q, K, Vt, Npad);
}

// ---------------------------------------------------------------- resident form
// One workgroup (8 waves) per (part, slot) walks token tiles; wave w keeps its 32
// output columns' weights for all 16 k-steps in registers (64 VGPRs, loaded once), so
// the GEMM reads only the x tile from LDS and nothing from L2.  The next tile's x rows
// arrive by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction, XOR swizzle
// applied to the source addresses) into the other of two buffers while this tile is
// computed and written.  Grid: per XCD `slots` x NPART workgroups; the parts of one
// token tile run on one XCD at the same time (tile t -> XCD t % 8), so x is read from
// HBM once and from that XCD's L2 by the other parts.
typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ unsigned lds_addr(char* p) { return (unsigned)(uintptr_t)(lds_char*)p; }
// The `s_nop 0` is the SALU-write-M0 -> LDS-DMA-read-M0 wait state (gfx9 family): hipcc
// sets M0 for the "{m0}" operand with an s_mov_b32 placed directly in front of the
// statement and pads hazards only for instructions it models, not for asm.  Without it
// the DMA could take the previous piece's M0 and land 1 KiB in the wrong slot, depending
// on issue timing (run-to-run / co-scheduling dependent results: DESIGN.md §5, r03a).
__device__ __forceinline__ void dma16(const void* g, unsigned m0) {
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}

template <bool SWAP>
__device__ __forceinline__ void res_gemm(const bf16x8 (&wf)[16], const char* lds, f32x16 (&acc)[2]) {
    const int lane = threadIdx.x & 63, col = lane & 31, hh = lane >> 5;
    const char* xrow = lds + col * ROWB;
    const int sw = col & 15;
    bf16x8 xa[2], xb[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) xa[mt] = *reinterpret_cast<const bf16x8*>(xrow + 32 * mt * ROWB + ((hh ^ sw) << 4));
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
        bf16x8(&cur)[2] = (ks & 1) ? xb : xa;
        bf16x8(&nxt)[2] = (ks & 1) ? xa : xb;
        if (ks < 15) {
            const int cn = ((2 * (ks + 1) + hh) ^ sw) << 4;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) nxt[mt] = *reinterpret_cast<const bf16x8*>(xrow + 32 * mt * ROWB + cn);
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
            acc[mt] = SWAP ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[mt], wf[ks], acc[mt], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], cur[mt], acc[mt], 0, 0, 0);
    }
}

template <bool SELF>
__global__ __launch_bounds__(512) void k_lg_proj_res(const bf16_t* __restrict__ xcopy, int ldx,
                                                       const bf16_t* __restrict__ W, const float* __restrict__ bias,
                                                       const float* __restrict__ efac,
                                                       const uint8_t* __restrict__ live, bf16_t* __restrict__ Q,
                                                       bf16_t* __restrict__ K, bf16_t* __restrict__ Vt, int Npad,
                                                       int slots, int probe) {
    constexpr int N = SELF ? 768 : 512, NPART = SELF ? 3 : 2, R = 64;
    // per buffer: x tile (32 KiB; the output staging image overlays it), then for the
    // self block the tile's rotary factors cos / sin [64][32] f32 (8 KiB each)
    constexpr int XB = R * ROWB, BUF = XB + (SELF ? 2 * R * 32 * 4 : 0);
    // + the tile's R live bytes (LDS-DMA with the tile)
    __shared__ __attribute__((aligned(16))) char buf0[BUF + R];
    __shared__ __attribute__((aligned(16))) char buf1[BUF + R];
    __shared__ __attribute__((aligned(16))) float bias_l[256];  // this part's biases
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 31, hh = lane >> 5;
    const int xcd = (int)blockIdx.x & 7, j = (int)blockIdx.x >> 3;
    const int part = j % NPART, slot = j / NPART;
    const int ntiles = Npad / R, stride = 8 * slots;
    int t = xcd + 8 * slot;
    if (slot >= slots || t >= ntiles) return;
    const bool is_v = part == NPART - 1;
    if (threadIdx.x < 256) bias_l[threadIdx.x] = bias[256 * part + threadIdx.x];  // read after the loop-top barrier
    bf16x8 wf[16];
    {
        const bf16_t* wrow = W + (size_t)(256 * part + 32 * wave + col) * 16 + 8 * hh;
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) wf[ks] = ld16(wrow + (size_t)ks * N * 16);
    }
    // this wave's four 1 KiB DMA pieces of a tile: rows 8 w + 2 i + (lane >> 5), slot lane & 31
    const int drow = 8 * wave + (lane >> 5), dslot = lane & 31;
    auto issue = [&](int tile, char* buf) {
        const unsigned base = lds_addr(buf) + 4096 * wave;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = drow + 2 * i;
            dma16(xcopy + (size_t)(tile * R + row) * ldx + ((dslot ^ (row & 15)) * 8), base + 1024 * i);
        }
        if (probe & 4) return;
        // (the v part fetches them too: skipping that measured slower, 1.92 vs 1.71 ms at 2 M
        // tokens; probably the three parts of a tile then drift apart and lose the L2 reuse)
        if (SELF && !(probe & 8)) {  // the tile's 16 KiB factor block: two 1 KiB pieces per wave
#pragma unroll
            for (int i = 0; i < 2; ++i)
                dma16(efac + (size_t)tile * (R * 64) + (2 * wave + i) * 256 + 4 * lane,
                      lds_addr(buf) + XB + 1024 * (2 * wave + i));
        }
        if (wave == 0 && lane < R / 16) dma16(live + (size_t)tile * R + 16 * lane, lds_addr(buf) + BUF);
    };
    issue(t, buf0);
    for (int it = 0;; ++it) {
        char* cur = (it & 1) ? buf1 : buf0;
        char* nxt = (it & 1) ? buf0 : buf1;
        // this wave's DMA of tile t has landed: vector-memory operations retire in issue
        // order, and the only ones issued after that DMA are the previous tile's four
        // copy-out stores per lane, which may stay in flight (vmcnt counts stores too;
        // the epilogue issues no global load)
        if (it == 0) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        else __builtin_amdgcn_s_waitcnt(0x0F74);          // vmcnt(4)
        __syncthreads();  // ... and every other wave's
        const int tn = t + stride;
        if (tn < ntiles) issue(tn, nxt);
        f32x16 acc[2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[mt][i] = 0.f;
        if (!(probe & 1)) {
            if (is_v) res_gemm<true>(wf, cur, acc);
            else res_gemm<false>(wf, cur, acc);
        }
        __syncthreads();  // every wave has read the x tile
        const float* fc = reinterpret_cast<const float*>(cur + XB);
        if (!(probe & 2)) proj_epilogue<SELF, 2, true>(acc, is_v, part, t * R, R | ((probe & 16) << 12), cur, bias_l, fc,
                                     reinterpret_cast<const uint8_t*>(cur + BUF), Q, K, Vt, Npad);
        if (tn >= ntiles) break;
        t = tn;
    }
}

// ---------------------------------------------------------------- pipelined resident form
// The resident form with the epilogue of tile t - 1 issued INSIDE the GEMM of tile t:
// every wave's bias / rotary / mask / bf16 staging of the previous tile's accumulators is
// cut into 8 slices (4 column groups x 2 m-tiles), one after every second k-step, so the
// VALU work fills the MFMA gaps instead of running in a phase of its own (the serial form
// spends about as long in its epilogue as in its GEMM).  Three LDS buffers: tile t's x
// rows (GEMM), tile t - 1's staging image over its dead x rows (+ its factors / live
// bytes), tile t + 1's DMA.  Only the copy-out stays a phase of its own, after the
// staging barrier.  Results are those of k_lg_proj_res bit for bit (same accumulators,
// same epilogue arithmetic).
// Paired staging (MLG_PROJ_SWAP): lanes l and l + 32 hold the two 8-B halves of one 16-B
// chunk (q / k: head dims 8c..+3 and 8c+4..+7 of token r; v: tokens 8g..+3 and 8g+4..+7 of
// dim d).  slice_*_val packs a slice's 8 B; stage_pair takes the m-tile 0 and 1 halves,
// swaps lanes 32-63 of the first with lanes 0-31 of the second (v_permlane32_swap), so
// lane l < 32 holds m-tile 0's whole chunk and lane l + 32 m-tile 1's, and writes it as
// ONE ds_write_b128 into an image whose chunk c of row r sits at slot c ^ (r & 7).  LDS
// writes retire 128 B per cycle in lane order (b128: 8 lanes, bank = address mod 128 B),
// reads 256 B (b128: 16 lanes, mod 256 B): the 8 consecutive rows of a write group then
// hit 8 distinct 16-B slots mod 128, and the copy-out's b128 reads of 2 rows x 8 chunks 16
// distinct slots mod 256 -- both conflict-free (tools/lds_probe.hip, profiles/
// r05x_lds_calibration.txt; a (r >> 1) & 7 swizzle paid 2-way on every write, the b64
// writes of stage_off 4 conflict cycles each).
#ifndef MLG_PROJ_PAIR_SW
#define MLG_PROJ_PAIR_SW 0  // 1: the (r >> 1) & 7 swizzle (A/B only)
#endif
__device__ __forceinline__ int stage_pair_off(int h, int row, int c) {
    return (h * 64 + row) * 128 + ((c ^ ((MLG_PROJ_PAIR_SW ? row >> 1 : row) & 7)) << 4);
}
__device__ __forceinline__ void stage_pair(uint2 m0v, uint2 m1v, char* lds, int h, int row, int c) {
    const auto s0 = __builtin_amdgcn_permlane32_swap(m0v.x, m1v.x, false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(m0v.y, m1v.y, false, false);
    *reinterpret_cast<uint4*>(lds + stage_pair_off(h, row, c)) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
}

template <bool SELF>
__device__ __forceinline__ uint2 slice_qk_val(int g, int mt, const f32x16& a, const float* bias_l, const float* fc,
                                              const uint8_t* live_l) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 31, hh = lane >> 5;
    const int n = 32 * wave + 8 * g + 4 * hh;
    const float4 b = *reinterpret_cast<const float4*>(bias_l + n);
    const int r = 32 * mt + col;
    float x0 = a[4 * g] + b.x, x1 = a[4 * g + 1] + b.y, x2 = a[4 * g + 2] + b.z, x3 = a[4 * g + 3] + b.w;
    if (SELF) {  // as slice_qk
        const float4 cs = fac_tile(fc, r, (n & 63) >> 2);
        const float r0 = __fadd_rn(__fmul_rn(x0, cs.x), __fmul_rn(-x1, cs.z));
        const float r1 = __fadd_rn(__fmul_rn(x1, cs.x), __fmul_rn(x0, cs.z));
        const float r2 = __fadd_rn(__fmul_rn(x2, cs.y), __fmul_rn(-x3, cs.w));
        const float r3 = __fadd_rn(__fmul_rn(x3, cs.y), __fmul_rn(x2, cs.w));
        x0 = r0; x1 = r1; x2 = r2; x3 = r3;
    }
    const uint32_t keep = 0u - (uint32_t)(live_l[r] != 0);
    return make_uint2(pack_bf16x2(x0, x1) & keep, pack_bf16x2(x2, x3) & keep);
}
// q / k pair write of column group g: row 32 hh + col, chunk (32 wave + 8 g) / 8 of head h
__device__ __forceinline__ void stage_pair_qk(int g, uint2 m0v, uint2 m1v, char* lds) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 31, hh = lane >> 5;
    const int n = 32 * wave + 8 * g;
    stage_pair(m0v, m1v, lds, n >> 6, 32 * hh + col, (n & 63) >> 3);
}

__device__ __forceinline__ uint2 slice_v_val(int g, int mt, const f32x16& a, const float* bias_l,
                                             const uint8_t* live_l) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 31, hh = lane >> 5;
    const float b = bias_l[32 * wave + col];
    const int r = 32 * mt + 8 * g + 4 * hh;
    const uint32_t lv = *reinterpret_cast<const uint32_t*>(live_l + r);
    const float v0 = (lv & 0xff) ? a[4 * g] + b : 0.f;
    const float v1 = (lv & 0xff00) ? a[4 * g + 1] + b : 0.f;
    const float v2 = (lv & 0xff0000) ? a[4 * g + 2] + b : 0.f;
    const float v3 = (lv >> 24) ? a[4 * g + 3] + b : 0.f;
    return make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
}
// V^T pair write of token group g: row d, chunk g + 4 hh (tokens 32 hh + 8 g ..) of head h
__device__ __forceinline__ void stage_pair_v(int g, uint2 m0v, uint2 m1v, char* lds) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 31, hh = lane >> 5;
    const int n = 32 * wave + col;
    stage_pair(m0v, m1v, lds, n >> 6, n & 63, g + 4 * hh);
}

template <bool SELF>
__device__ __forceinline__ void slice_qk(int g, int mt, const f32x16& a, char* lds, const float* bias_l,
                                         const float* fc, const uint8_t* live_l) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 31, hh = lane >> 5;
    const int n = 32 * wave + 8 * g + 4 * hh, h = n >> 6, d = n & 63;
    const float4 b = *reinterpret_cast<const float4*>(bias_l + n);
    const int r = 32 * mt + col;
    float x0 = a[4 * g] + b.x, x1 = a[4 * g + 1] + b.y, x2 = a[4 * g + 2] + b.z, x3 = a[4 * g + 3] + b.w;
    if (SELF) {  // as proj_epilogue's resident form
        const float4 cs = fac_tile(fc, r, (n & 63) >> 2);  // cos j, cos j + 1, sin j, sin j + 1
        const float r0 = __fadd_rn(__fmul_rn(x0, cs.x), __fmul_rn(-x1, cs.z));
        const float r1 = __fadd_rn(__fmul_rn(x1, cs.x), __fmul_rn(x0, cs.z));
        const float r2 = __fadd_rn(__fmul_rn(x2, cs.y), __fmul_rn(-x3, cs.w));
        const float r3 = __fadd_rn(__fmul_rn(x3, cs.y), __fmul_rn(x2, cs.w));
        x0 = r0; x1 = r1; x2 = r2; x3 = r3;
    }
    // branch-free mask: a branch here would end the basic block and with it the
    // scheduler's freedom to interleave this slice with the GEMM's MFMAs
    const uint32_t keep = 0u - (uint32_t)(live_l[r] != 0);
    *reinterpret_cast<uint2*>(lds + stage_off<64>(h, r, d)) =
        make_uint2(pack_bf16x2(x0, x1) & keep, pack_bf16x2(x2, x3) & keep);
}

__device__ __forceinline__ void slice_v(int g, int mt, const f32x16& a, char* lds, const float* bias_l,
                                        const uint8_t* live_l) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 31, hh = lane >> 5;
    const int n = 32 * wave + col, h = n >> 6, d = n & 63;
    const float b = bias_l[n];
    const int r = 32 * mt + 8 * g + 4 * hh;
    const uint32_t lv = *reinterpret_cast<const uint32_t*>(live_l + r);
    const float v0 = (lv & 0xff) ? a[4 * g] + b : 0.f;
    const float v1 = (lv & 0xff00) ? a[4 * g + 1] + b : 0.f;
    const float v2 = (lv & 0xff0000) ? a[4 * g + 2] + b : 0.f;
    const float v3 = (lv >> 24) ? a[4 * g + 3] + b : 0.f;
    *reinterpret_cast<uint2*>(lds + stage_off<64>(h, d, r)) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
}

// acc_new = GEMM of the x tile in `xl`; with STAGE, slice i of the previous tile's
// staging (acc_old into `sl`) after k-step 2 i.
template <bool SELF, bool IS_V, bool STAGE>
__device__ __forceinline__ void pipe_gemm(const bf16x8 (&wf)[16], const char* xl, f32x16 (&acc)[2],
                                          const f32x16 (&old)[2], char* sl, const float* bias_l, const float* fc,
                                          const uint8_t* live_l) {
    const int lane = threadIdx.x & 63, col = lane & 31, hh = lane >> 5;
    const char* xrow = xl + col * ROWB;
    const int sw = col & 15;
    bf16x8 xa[2], xb[2];
    uint2 pend = make_uint2(0u, 0u);  // MLG_PROJ_SWAP: m-tile 0's half of the pending pair
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) xa[mt] = *reinterpret_cast<const bf16x8*>(xrow + 32 * mt * ROWB + ((hh ^ sw) << 4));
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
        bf16x8(&cur)[2] = (ks & 1) ? xb : xa;
        bf16x8(&nxt)[2] = (ks & 1) ? xa : xb;
        if (ks < 15) {
            const int cn = ((2 * (ks + 1) + hh) ^ sw) << 4;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) nxt[mt] = *reinterpret_cast<const bf16x8*>(xrow + 32 * mt * ROWB + cn);
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
            acc[mt] = IS_V ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[mt], wf[ks], acc[mt], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], cur[mt], acc[mt], 0, 0, 0);
        if (STAGE && !(ks & 1)) {
            const int g = ks >> 2, mt = (ks >> 1) & 1;
            if (MLG_PROJ_SWAP) {  // m-tile 0's half at ks = 4 g, the pair write at 4 g + 2
                const uint2 v = IS_V ? slice_v_val(g, mt, old[mt], bias_l, live_l)
                                     : slice_qk_val<SELF>(g, mt, old[mt], bias_l, fc, live_l);
                if (mt == 0) {
                    pend = v;
                } else if (IS_V) {
                    stage_pair_v(g, pend, v, sl);
                } else {
                    stage_pair_qk(g, pend, v, sl);
                }
            } else if (IS_V) {
                slice_v(g, mt, old[mt], sl, bias_l, live_l);
            } else {
                slice_qk<SELF>(g, mt, old[mt], sl, bias_l, fc, live_l);
            }
        }
    }
}

// copy-out of a staged 64-token tile (proj_epilogue's second half)
__device__ __forceinline__ void copy_out64(bool is_v, int part, int m0, const char* lds, bf16_t* __restrict__ Q,
                                           bf16_t* __restrict__ K, bf16_t* __restrict__ Vt, int Npad) {
    bf16_t* dst = is_v ? Vt : (part == 0 ? Q : K);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int L = p * 512 + threadIdx.x, h = L / 512, row = (L >> 3) & 63, c = L & 7;
        *reinterpret_cast<uint4*>(dst + ((size_t)h * Npad + m0 + row) * 64 + c * 8) =
            *reinterpret_cast<const uint4*>(lds + (MLG_PROJ_SWAP ? stage_pair_off(h, row, c) : stage_off<64>(h, row, 8 * c)));
    }
}

template <bool SELF, bool IS_V>
__device__ __forceinline__ void pipe_tiles(const bf16x8 (&wf)[16], char* ring, const float* bias_l,
                                           const bf16_t* __restrict__ xcopy, int ldx, const float* __restrict__ efac,
                                           const uint8_t* __restrict__ live,
                                           bf16_t* __restrict__ Q, bf16_t* __restrict__ K, bf16_t* __restrict__ Vt,
                                           int Npad, int part, int t0, int stride, int ntiles) {
    constexpr int R = 64, XB = R * ROWB, BUF = XB + (SELF ? 2 * R * 32 * 4 : 0), SLOT = BUF + 256;
    auto bufs = [&](int i) { return ring + i * SLOT; };
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int drow = 8 * wave + (lane >> 5), dslot = lane & 31;
    auto issue = [&](int tile, char* buf) {
        const unsigned base = lds_addr(buf) + 4096 * wave;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = drow + 2 * i;
            dma16(xcopy + (size_t)(tile * R + row) * ldx + ((dslot ^ (row & 15)) * 8), base + 1024 * i);
        }
        if (SELF) {  // the tile's 16 KiB factor block: two 1 KiB pieces per wave
#pragma unroll
            for (int i = 0; i < 2; ++i)
                dma16(efac + (size_t)tile * (R * 64) + (2 * wave + i) * 256 + 4 * lane,
                      lds_addr(buf) + XB + 1024 * (2 * wave + i));
        }
        if (wave == 0 && lane < R / 16) dma16(live + (size_t)tile * R + 16 * lane, lds_addr(buf) + BUF);
    };
    f32x16 acc0[2], acc1[2];  // the GEMM's and the staged tile's, alternating (compile-time roles)
    issue(t0, bufs(0));
    int t = t0, tp = -1, it = 0;  // tile in the GEMM, tile being staged (-1: none)
    // one iteration; PAR = it & 1 picks the accumulator roles
    auto step = [&](f32x16 (&an)[2], const f32x16 (&ao)[2]) -> bool {
        const int bx = it % 3, bp = (it + 2) % 3, bn = (it + 1) % 3;
        // tile t's DMA has landed (only the previous iteration's 4 copy-out stores per lane
        // were issued after it; none in the first two iterations)
        if (it < 2) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        else __builtin_amdgcn_s_waitcnt(0x0F74);         // vmcnt(4)
        __syncthreads();  // every wave's DMA; every wave's copy-out reads of buffer bn
        const int tn = t + stride;
        if (tn < ntiles) issue(tn, bufs(bn));
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int i = 0; i < 16; ++i) an[mt][i] = 0.f;
        char* sl = bufs(bp);
        const float* fc = reinterpret_cast<const float*>(sl + XB);
        if (tp >= 0) {
            pipe_gemm<SELF, IS_V, true>(wf, bufs(bx), an, ao, sl, bias_l, fc,
                                        reinterpret_cast<const uint8_t*>(sl + BUF));
            __syncthreads();  // staging written
            copy_out64(IS_V, part, tp * R, sl, Q, K, Vt, Npad);
        } else {
            pipe_gemm<SELF, IS_V, false>(wf, bufs(bx), an, ao, sl, bias_l, fc,
                                         reinterpret_cast<const uint8_t*>(sl + BUF));
        }
        tp = t;
        ++it;
        if (tn >= ntiles) {  // the last tile: its staging alone
            __syncthreads();  // every wave has read its x rows
            char* sx = bufs(bx);
            const float* fx = reinterpret_cast<const float*>(sx + XB);
            const uint8_t* lx = reinterpret_cast<const uint8_t*>(sx + BUF);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (MLG_PROJ_SWAP) {
                    if (i & 1) continue;
                    const int g = i >> 1;
                    if (IS_V)
                        stage_pair_v(g, slice_v_val(g, 0, an[0], bias_l, lx), slice_v_val(g, 1, an[1], bias_l, lx), sx);
                    else
                        stage_pair_qk(g, slice_qk_val<SELF>(g, 0, an[0], bias_l, fx, lx),
                                      slice_qk_val<SELF>(g, 1, an[1], bias_l, fx, lx), sx);
                } else if (IS_V) {
                    slice_v(i >> 1, i & 1, an[i & 1], sx, bias_l, lx);
                } else {
                    slice_qk<SELF>(i >> 1, i & 1, an[i & 1], sx, bias_l, fx, lx);
                }
            }
            __syncthreads();
            copy_out64(IS_V, part, tp * R, sx, Q, K, Vt, Npad);
            return true;
        }
        t = tn;
        return false;
    };
    for (;;) {
        if (step(acc0, acc1)) return;
        if (step(acc1, acc0)) return;
    }
}

template <bool SELF>
__global__ __launch_bounds__(512) void k_lg_proj_pipe(const bf16_t* __restrict__ xcopy, int ldx,
                                                        const bf16_t* __restrict__ W, const float* __restrict__ bias,
                                                        const float* __restrict__ efac,
                                                        const uint8_t* __restrict__ live, bf16_t* __restrict__ Q,
                                                        bf16_t* __restrict__ K, bf16_t* __restrict__ Vt, int Npad,
                                                        int slots) {
    constexpr int N = SELF ? 768 : 512, NPART = SELF ? 3 : 2, R = 64;
    constexpr int SLOT = R * ROWB + (SELF ? 2 * R * 32 * 4 : 0) + 256;  // x, factors, live bytes (pipe_tiles)
    __shared__ __attribute__((aligned(16))) char ring[3 * SLOT];
    __shared__ __attribute__((aligned(16))) float bias_l[256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 31, hh = lane >> 5;
    const int xcd = (int)blockIdx.x & 7, j = (int)blockIdx.x >> 3;
    const int part = j % NPART, slot = j / NPART;
    const int ntiles = Npad / R, stride = 8 * slots;
    const int t0 = xcd + 8 * slot;
    if (slot >= slots || t0 >= ntiles) return;
    if (threadIdx.x < 256) bias_l[threadIdx.x] = bias[256 * part + threadIdx.x];  // read after the loop-top barrier
    bf16x8 wf[16];
    {
        const bf16_t* wrow = W + (size_t)(256 * part + 32 * wave + col) * 16 + 8 * hh;
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) wf[ks] = ld16(wrow + (size_t)ks * N * 16);
    }
    if (part == NPART - 1)
        pipe_tiles<SELF, true>(wf, ring, bias_l, xcopy, ldx, efac, live, Q, K, Vt, Npad, part, t0, stride, ntiles);
    else
        pipe_tiles<SELF, false>(wf, ring, bias_l, xcopy, ldx, efac, live, Q, K, Vt, Npad, part, t0, stride,
                                ntiles);
}

}  // namespace

int mlg_lg_proj(bool self_block, const bf16_t* xcopy, int ldx, const bf16_t* W, const float* bias, const float* efac,
                const uint8_t* live, bf16_t* Q, bf16_t* K, bf16_t* Vt, int Npad, hipStream_t s) {
    if (Npad <= 0 || (Npad % 64) || ldx < 256 || (ldx % 8)) return MLG_EINVAL;
    // Build-time A/B knob: MLG_PROJ_MT = 32-token m-tiles per workgroup (2: 64 tokens, 4: 128).
    // 128-token tiles halve the weight bytes per FLOP but measured 2-7 % slower on one
    // box (tools/archive/gpu_ab_ffn_proj.sh: self 2.39 vs 2.35 ms, cross 1.27 vs 1.19 ms at 2 M
    // tokens): the weight stream is not what bounds this kernel.
    constexpr int mt = MLG_PROJ_MT == 4 ? 4 : 2;
    // default: the weights-resident persistent form; MLG_PROJ_RES=0 builds the tiled form
    if (MLG_PROJ_RES) {
        static const int cus = [] {
            int dev = 0, c = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 8)
                return 256;
            return c;
        }();
        // timing-probe builds only (MLG_PROJ_PROBE, results wrong; 0 in the product): 1 no GEMM, 2 no epilogue, 4 no DMA, 8 no factor DMA,
        // 16 no copy-out stores
        constexpr int probe = MLG_PROJ_PROBE;
        const int npart = self_block ? 3 : 2, ntiles = Npad / 64;
        // one workgroup per CU (256 VGPRs, 64-96 KiB LDS), `slots` part-groups per XCD
        const int slots = std::max(1, std::min((cus / 8) / npart, (ntiles + 7) / 8));
        const unsigned grid = (unsigned)(8 * slots * npart);
        if (MLG_PROJ_PIPE && !probe) {
            if (self_block)
                hipLaunchKernelGGL(k_lg_proj_pipe<true>, dim3(grid), dim3(512), 0, s, xcopy, ldx, W, bias, efac,
                                   live, Q, K, Vt, Npad, slots);
            else
                hipLaunchKernelGGL(k_lg_proj_pipe<false>, dim3(grid), dim3(512), 0, s, xcopy, ldx, W, bias,
                                   (const float*)nullptr, live, Q, (bf16_t*)nullptr, Vt, Npad,
                                   slots);
            MLG_LAUNCH_CHECK();
            return MLG_OK;
        }
        if (self_block)
            hipLaunchKernelGGL(k_lg_proj_res<true>, dim3(grid), dim3(512), 0, s, xcopy, ldx, W, bias, efac, live,
                               Q, K, Vt, Npad, slots, probe);
        else
            hipLaunchKernelGGL(k_lg_proj_res<false>, dim3(grid), dim3(512), 0, s, xcopy, ldx, W, bias,
                               (const float*)nullptr, live, Q, (bf16_t*)nullptr, Vt, Npad,
                               slots, probe);
        MLG_LAUNCH_CHECK();
        return MLG_OK;
    }
    const int R = 32 * mt;
    const unsigned grid = (unsigned)((((long)((Npad + R - 1) / R) * (self_block ? 3 : 2)) + 7) & ~7L);
    if (self_block) {
        if (mt == 4)
            hipLaunchKernelGGL((k_lg_proj<true, 4>), dim3(grid), dim3(512), 0, s, xcopy, ldx, W, bias, efac,
                               live, Q, K, Vt, Npad);
        else
            hipLaunchKernelGGL((k_lg_proj<true, 2>), dim3(grid), dim3(512), 0, s, xcopy, ldx, W, bias, efac,
                               live, Q, K, Vt, Npad);
    } else {
        if (mt == 4)
            hipLaunchKernelGGL((k_lg_proj<false, 4>), dim3(grid), dim3(512), 0, s, xcopy, ldx, W, bias,
                               (const float*)nullptr, live, Q, (bf16_t*)nullptr, Vt, Npad);
        else
            hipLaunchKernelGGL((k_lg_proj<false, 2>), dim3(grid), dim3(512), 0, s, xcopy, ldx, W, bias,
                               (const float*)nullptr, live, Q, (bf16_t*)nullptr, Vt, Npad);
    }
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}
