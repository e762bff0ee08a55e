// Fused tail of a LightGlue transformer block (SelfBlock / CrossBlock of upstream
// LightGlue, called by LightGlue._detect_and_match_native,
// scripts/semantic_gating/geometric_verification.py:263-312):
//
//   msg = out_proj(ctx)                               (to_out for the cross block)
//   x  += Linear2( GELU( LayerNorm( Linear1( [x | msg] ) ) ) )
//
// in ONE kernel per 64-token tile.  Unfused, this tail moved ~10.5 KB of HBM per token
// (ctx, msg, the f32 FFN hidden, its bf16 GELU output, x twice); fused, the
// concatenation, the hidden and the GELU output never leave LDS: 3.5 KB per token (ctx
// and the bf16 copy of x in; the f32 residual read, updated and written; the new bf16
// copy of x, which the next block's projections read, written).
//
// One workgroup = 4 waves = 64 token rows, two workgroups per CU, so one workgroup's
// HBM phases (tile in, residual out) overlap the other's MFMAs.  LDS holds the tile's
// [x | ctx] as bf16 [64][512] (XOR-swizzled 16-B chunks); the three GEMMs run as
// C^T = W . T^T with v_mfma_f32_32x32x16_bf16 (W fragments from global/L2, k-step-major
// packed, in a register ring four k-steps ahead; token fragments from LDS,
// double-buffered one k-step ahead), each wave owning a slice of the output columns for
// all 64 rows:
//   1. msg  : wave w -> cols [64w, 64w+64) of 256   (K = 256 over the ctx half);
//             msg + bias, bf16, overwrites the ctx half in LDS
//   2. ffn1 : wave w -> cols [128w, 128w+128) of 512 (K = 512 over [x | msg]);
//             + bias, LayerNorm(512, eps 1e-5) statistics reduced lane -> half-wave ->
//             4 waves through LDS (two passes: mean, then centred variance), GELU (erf
//             form, common.h gelu_poly2),
//             bf16, overwrites [x | msg] in LDS
//   3. ffn2 : wave w -> cols [64w, 64w+64) of 256   (K = 512);
//             x += acc + bias (f32), bf16 copy of x written for the next projections.
// The accumulator of the transposed product gives each lane 4 consecutive output
// columns of one token: LayerNorm sums are lane-local up to one cross-half exchange,
// and every epilogue store is a 4-wide vector.
#include <stdlib.h>

#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int ROWB = 1024;  // LDS bytes per token row: 512 bf16

// 16-B chunk c of row r at slot c ^ (r & 15): the 16 lanes of each ds_read_b128 lane
// group (rows {0-3,12-15,20-27} + 32 k, one chunk) then hit 16 distinct bank quads.
__device__ __forceinline__ int cat_off(int row, int chunk) { return row * ROWB + ((chunk ^ (row & 15)) << 4); }

// Epilogue writes into [x | msg] / the GELU tile (MLG_FFN_STAGE_W, MT = 2): lanes l and
// l + 32 hold the two 8-B halves of one 16-B chunk (rows col and 32 + col in m-tiles 0 / 1);
// a v_permlane32_swap gives lane l < 32 m-tile 0's whole chunk and lane l + 32 m-tile 1's,
// written as one b128.  LDS writes retire 128 B per cycle in lane order (b128: 8 lanes,
// banks modulo 128 B; profiles/r05x_lds_calibration.txt): 8 consecutive rows at slots
// chunk ^ (r & 15) are distinct modulo 128 B -- the per-half b64 writes paid 2-way.
#ifndef MLG_FFN_STAGE_W
#define MLG_FFN_STAGE_W 1
#endif
__device__ __forceinline__ void cat_pair_write(char* lds, int chunk, uint2 m0v, uint2 m1v) {
    const int lane = threadIdx.x & 63, col = lane & 31, hh = lane >> 5;
    const auto s0 = __builtin_amdgcn_permlane32_swap(m0v.x, m1v.x, false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(m0v.y, m1v.y, false, false);
    *reinterpret_cast<uint4*>(lds + cat_off(32 * hh + col, chunk)) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
}

__device__ __forceinline__ bf16x8 ld16(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// The tile's token rows are read once and the residual written once per block: they go
// through non-temporal (streaming) accesses so they do not evict the block's weights,
// which every tile of the launch re-reads from L2 (same-box A/B: 385.6 -> 379.6 ms of FFN
// per 4096-pair call, profiles/r03ac_ab_ffn_nontemporal.txt).
#ifndef MLG_FFN_NT
#define MLG_FFN_NT 1
#endif
// Launch form, fixed per build (A/B arms are separate builds loaded through
// tools/ab_run.py): MLG_FFN_GRID = workgroups per CU of a persistent grid (0: one
// workgroup per tile), MLG_FFN_ROWS = token rows per workgroup (64: 4 waves, 128: 8).
#ifndef MLG_FFN_GRID
#define MLG_FFN_GRID 0
#endif
#ifndef MLG_FFN_ROWS
#define MLG_FFN_ROWS 64
#endif
#ifndef MLG_FFN_XR_WAIT
#define MLG_FFN_XR_WAIT 0
#endif
// LayerNorm rstd: 1 = the bare v_rsq_f32 (product), 0 = rsqrtf with its denormal fix-up,
// 2 = bare + 5 wait states (probe arm).  Under hipcc's SLP pass form 0 packed the two
// m-tiles' fix-ups into one v_pk_mul_f32 reading both v_rsq_f32 results one wait state
// later, which gave co-scheduling dependent rstd (DESIGN.md §5, round-4 FFN probe).
#ifndef MLG_FFN_RSQ
#define MLG_FFN_RSQ 1
#endif
#ifndef MLG_FFN_RING1
#define MLG_FFN_RING1 2
#endif
// timing-probe builds only (results wrong; 0 in the product), bits drop one phase each:
// 1 GELU polynomial (the normalised value passes), 2 LayerNorm statistics (mean 0,
// rstd 1), 4 msg GEMM, 8 ffn1 GEMM, 16 ffn2 GEMM, 32 residual row pass, 64 tile load
#ifndef MLG_FFN_PROBE
#define MLG_FFN_PROBE 0
#endif
// Phase stagger of the two co-resident workgroups of a CU: every tile runs the same
// sequence (GEMM, VALU-heavy LayerNorm + GELU, GEMM), so two workgroups that start
// together stay in step and meet in the same phase.  The second resident set (mode 1:
// blocks [n_cu, 2 n_cu); mode 2: odd blocks below 2 n_cu) first sleeps MLG_FFN_STAGGER x
// 127 x 64 cycles; later tiles inherit the offset.  Arithmetic unchanged.
#ifndef MLG_FFN_STAGGER
#define MLG_FFN_STAGGER 0
#endif
#ifndef MLG_FFN_STAGGER_MODE
#define MLG_FFN_STAGGER_MODE 1
#endif
#ifndef MLG_FFN_RING2
#define MLG_FFN_RING2 4
#endif
// Phase timestamps (probe builds, MLG_FFN_TRACE=1): s_memtime at the phase boundaries of
// every workgroup's tile, with the wave's HW_ID / XCC_ID, read by mlg_dbg_ffn_trace
// (tools/ffn_trace.py).  0 in the product.
#ifndef MLG_FFN_TRACE
#define MLG_FFN_TRACE 0
#endif
[[maybe_unused]] constexpr int FFN_TRACE_WGS = 65536, FFN_TRACE_W = 12;
#if MLG_FFN_TRACE
__device__ unsigned long long g_ffn_trace[FFN_TRACE_WGS * FFN_TRACE_W];
#define FFN_T(i) tt[i] = __builtin_amdgcn_s_memtime()
#else
#define FFN_T(i) (void)0
#endif
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
__device__ __forceinline__ uint4 stream_ld(const uint4* p) {
#if MLG_FFN_NT
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ float4 stream_ld(const float4* p) {
#if MLG_FFN_NT
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ void stream_st(float4* p, const float4& v) {
#if MLG_FFN_NT
    __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(p));
#else
    *p = v;
#endif
}

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }
// log(sigmoid(x)) = min(x, 0) - log1p(exp(-|x|))  (torch's stable form)
__device__ __forceinline__ float logsigmoid_f(float x) { return fminf(x, 0.f) - log1pf(expf(-fabsf(x))); }

// acc[t][mt] += W[n0 + 32 t + i][k] * T[32 mt + j][k] over K = 64 * nkb, with T the LDS
// tile starting at 16-B chunk `chunk0` (k-step ks at chunk chunk0 + 2 ks + hh).  W is
// packed k-step-major, [K/16][N][16] bf16 (mlgate.lightglue.pack_kstep), so the 32 rows
// x 32 B a wave reads per k-step are one contiguous 1 KiB: every fetched line is
// consumed by the instruction that fetched it.  W fragments live in a 4-step register
// ring (slot s refilled with step ks + 4 as soon as step ks's MFMAs have issued); token
// fragments are read one k-step ahead into the other half of a double buffer.  Loads
// past the last step re-read the last step (no branches, so the waitcnt pass counts
// the in-flight loads exactly); addresses are recomputed per call, not hoisted.
template <int NT, int MT, int RING = 4>
__device__ __forceinline__ void gemm_phase(const bf16_t* __restrict__ W, int N, int n0, int nkb, int chunk0,
                                           const char* lds, f32x16 (&acc)[NT][MT]) {
    const int lane = threadIdx.x & 63, col = lane & 31, hh = lane >> 5;
    const size_t step = (size_t)N * 16;
    const int last = 4 * nkb - 1;
    const bf16_t* wrow[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) wrow[t] = W + (size_t)(n0 + 32 * t + col) * 16 + 8 * hh;
    const char* xrow = lds + col * ROWB;  // + 32 mt rows per m-tile
    const int sw = col & 15;             // = row & 15 for every m-tile
    bf16x8 wf[NT][RING], xa[MT], xb[MT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int s = 0; s < RING; ++s) wf[t][s] = ld16(wrow[t] + s * step);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
        xa[mt] = *reinterpret_cast<const bf16x8*>(xrow + 32 * mt * ROWB + (((chunk0 + hh) ^ sw) << 4));
#pragma unroll 1
    for (int kb = 0; kb < 4 * nkb / RING; ++kb) {
#pragma unroll
        for (int s = 0; s < RING; ++s) {
            const int ks = RING * kb + s;
            const int cn = ((chunk0 + 2 * min(ks + 1, last) + hh) ^ sw) << 4;
            bf16x8(&cur)[MT] = (s & 1) ? xb : xa;
            bf16x8(&nxt)[MT] = (s & 1) ? xa : xb;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) nxt[mt] = *reinterpret_cast<const bf16x8*>(xrow + 32 * mt * ROWB + cn);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    acc[t][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[t][s], cur[mt], acc[t][mt], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < NT; ++t) wf[t][s] = ld16(wrow[t] + min(ks + RING, last) * step);
            // pin the refill here: left alone, the scheduler sinks it next to its use
            // (minimising live ranges) and every step waits on a fresh L2 round trip
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

template <int NT, int MT>
__device__ __forceinline__ void zero(f32x16 (&acc)[NT][MT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[t][mt][i] = 0.f;
}

// relu != 0: SuperGlue's MLP (BatchNorm folded into Wf1 / bf1 on the host, ReLU, no
// LayerNorm) instead of LightGlue's LayerNorm + GELU (superglue.hip)
//
// PERSIST = false (default): one workgroup per 64-row tile, 228 VGPRs, no scratch.
// PERSIST = true (MLG_FFN_GRID = workgroups per CU): the grid walks the tiles with stride
// gridDim.x; the compiler hoists lane addresses out of the tile loop and spills 436 B
// per lane around it: 3.66 vs 2.94 ms per 2 M-token launch and 4.29 vs 3.20 s of FFN per
// bench step on one box (tools/archive/gpu_ab_ffn_proj.sh), so it is off.
// R token rows per workgroup of NW waves: <64, 4> (two workgroups per CU) or <128, 8>
// (one per CU: every weight fragment fetched from L2 feeds twice the MFMAs).
//
// LOFTR: the tail of a LoFTREncoderLayer (kornia loftr/loftr_module/transformer.py, the
// reference's LoFTR matcher, geometric_verification.py:458-526) on the same three GEMMs:
//   msg = norm1(merge(attn));  x += norm2(mlp(cat[x, msg]))   (mlp: Linear, ReLU, Linear)
// no biases; norm1 (LayerNorm 256) in the msg epilogue, norm2 in the final row pass;
// LayerNorm affine from ln_g / ln_b = [norm1 (256) | norm2 (256)].
// RELU (SuperGlue's MLP) is a template argument, not a kernel argument: a run-time flag
// left a uniform branch around every 4-column group of the GELU epilogue, and each
// basic block held just two dependent 13-step Horner chains (the scheduler cannot
// interleave groups across blocks).
template <bool PERSIST, int R, int NW, bool LOFTR = false, bool RELU = false>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void k_lg_ffn(const bf16_t* __restrict__ ctx, float* __restrict__ X,
                                                  bf16_t* __restrict__ xcopy, int ldc, int M, mlg_lg_block_i w,
                                                  mlg_lg_conf_i cf) {
    constexpr bool relu = LOFTR || RELU;
#if MLG_FFN_TRACE
    unsigned long long tt[10] = {};
#endif
    FFN_T(0);
    constexpr int MT = R / 32, NT1 = 256 / NW / 32, NT2 = 512 / NW / 32, NTH = 64 * NW;
    constexpr int RING = NW == 8 ? 8 : MLG_FFN_RING2;  // weight k-steps in flight per wave (ffn1)
    // ring of the msg / ffn2 phases (NT1 column tiles, half the MFMAs per k-step of ffn1).
    // Same-box sweep (profiles/r03an_ab_ffn_ring.txt, identical matches in every arm): msg /
    // ffn2 ring 2 / 4 / 8 / 16 -> 374 / 376 / 379 / 432 ms of FFN per 4096-pair call, ffn1
    // ring 2 / 4 / 8 -> 382 / 376 / 506 ms: more loads in flight only cost, so the L2
    // latency of the weight stream is covered already.
    constexpr int RING1 = NW == 8 ? 8 : MLG_FFN_RING1;
    __shared__ __attribute__((aligned(16))) char lds[R * ROWB];
    __shared__ float red[2][NW][R];
    // biases and LayerNorm affine, staged in LDS: epilogue reads never wait on VMEM
    // behind the in-flight weight loads
    __shared__ __attribute__((aligned(16))) float prm[256 + 512 + 512 + 512 + 256];
    float* s_bout = prm;
    float* s_bf1 = prm + 256;
    float* s_lng = prm + 768;
    float* s_lnb = prm + 1280;
    float* s_bf2 = prm + 1792;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 31, hh = lane >> 5;
    for (int i = tid; i < 512; i += NTH) {
        s_bf1[i] = LOFTR ? 0.f : w.bf1[i];
        s_lng[i] = (relu && !LOFTR) ? 1.f : w.ln_g[i];
        s_lnb[i] = (relu && !LOFTR) ? 0.f : w.ln_b[i];
        if (i < 256) {
            s_bout[i] = LOFTR ? 0.f : w.bout[i];
            s_bf2[i] = LOFTR ? 0.f : w.bf2[i];
        }
    }
    if constexpr (MLG_FFN_STAGGER > 0 && !PERSIST) {
        const unsigned b = blockIdx.x;
        const bool late = MLG_FFN_STAGGER_MODE == 1 ? (b >= 256u && b < 512u) : (b < 512u && (b & 1u));
        if (late)
            for (int i = 0; i < MLG_FFN_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
    }
    const int ntiles = (M + R - 1) / R;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int m0 = tile * R;
        // 0. tile -> LDS: the bf16 copy of x (written by the previous block) into chunks
        //    0..31, ctx into chunks 32..63; 32 lanes x 16 B = one 512-B row per half-wave,
        //    rows clamped to M - 1 (never stored)
        if (!(MLG_FFN_PROBE & 64)) {
            constexpr int PASSES = R / (2 * NW);
            uint4 rx[PASSES], rc[PASSES];
            const int c = lane & 31;
    #pragma unroll
            for (int i = 0; i < PASSES; ++i) {
                const int row = 2 * NW * i + 2 * wave + hh;
                const size_t gr = (size_t)min(m0 + row, M - 1);
                rx[i] = stream_ld(reinterpret_cast<const uint4*>(xcopy + gr * ldc + c * 8));
                rc[i] = stream_ld(reinterpret_cast<const uint4*>(ctx + gr * 256 + c * 8));
            }
    #pragma unroll
            for (int i = 0; i < PASSES; ++i) {
                const int row = 2 * NW * i + 2 * wave + hh;
                *reinterpret_cast<uint4*>(lds + cat_off(row, c)) = rx[i];
                *reinterpret_cast<uint4*>(lds + cat_off(row, 32 + c)) = rc[i];
            }
        }
        __syncthreads();
        FFN_T(1);

        // 1. msg = ctx . Wout^T + bout  -> bf16 over the ctx half
        {
            f32x16 acc[NT1][MT];
            zero(acc);
            if (!(MLG_FFN_PROBE & 4)) gemm_phase<NT1, MT, RING1>(w.Wout, 256, 32 * NT1 * wave, 4, 32, lds, acc);
            __syncthreads();  // every wave has read the ctx half
            FFN_T(2);
            float mean1[MT], rstd1[MT];
            if constexpr (LOFTR) {
                // norm1 over the 256 msg columns of each row: lane -> half-wave -> waves
                // through LDS, two passes (mean, then centred variance) as torch
    #pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    float sum = 0.f;
    #pragma unroll
                    for (int t = 0; t < NT1; ++t)
    #pragma unroll
                        for (int i = 0; i < 16; ++i) sum += acc[t][mt][i];
                    sum += __shfl_xor(sum, 32, 64);
                    if (hh == 0) red[0][wave][32 * mt + col] = sum;
                }
                __syncthreads();
    #pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    float sum = 0.f;
    #pragma unroll
                    for (int v = 0; v < NW; ++v) sum += red[0][v][32 * mt + col];
                    mean1[mt] = sum * (1.0f / 256.0f);
                    float q = 0.f;
    #pragma unroll
                    for (int t = 0; t < NT1; ++t)
    #pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            const float d = acc[t][mt][i] - mean1[mt];
                            q += d * d;
                        }
                    q += __shfl_xor(q, 32, 64);
                    if (hh == 0) red[1][wave][32 * mt + col] = q;
                }
                __syncthreads();
    #pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    float q = 0.f;
    #pragma unroll
                    for (int v = 0; v < NW; ++v) q += red[1][v][32 * mt + col];
                    rstd1[mt] = 1.0f / sqrtf(q * (1.0f / 256.0f) + 1e-5f);
                }
            }
    #pragma unroll
            for (int t = 0; t < NT1; ++t)
    #pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int n = 32 * NT1 * wave + 32 * t + 8 * g + 4 * hh;
                    const float4 b = *reinterpret_cast<const float4*>(s_bout + n);
                    uint2 pk[MT];
    #pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        const f32x16& a = acc[t][mt];
                        float y0, y1, y2, y3;
                        if constexpr (LOFTR) {
                            const float4 lg = *reinterpret_cast<const float4*>(s_lng + n);
                            const float4 lb = *reinterpret_cast<const float4*>(s_lnb + n);
                            y0 = (a[4 * g] - mean1[mt]) * rstd1[mt] * lg.x + lb.x;
                            y1 = (a[4 * g + 1] - mean1[mt]) * rstd1[mt] * lg.y + lb.y;
                            y2 = (a[4 * g + 2] - mean1[mt]) * rstd1[mt] * lg.z + lb.z;
                            y3 = (a[4 * g + 3] - mean1[mt]) * rstd1[mt] * lg.w + lb.w;
                        } else {
                            y0 = a[4 * g] + b.x;
                            y1 = a[4 * g + 1] + b.y;
                            y2 = a[4 * g + 2] + b.z;
                            y3 = a[4 * g + 3] + b.w;
                        }
                        pk[mt] = make_uint2(pack_bf16x2(y0, y1), pack_bf16x2(y2, y3));
                    }
                    if constexpr (MLG_FFN_STAGE_W && MT == 2) {
                        cat_pair_write(lds, 32 + n / 8, pk[0], pk[MT - 1]);
                    } else {
    #pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
                            *reinterpret_cast<uint2*>(lds + cat_off(32 * mt + col, 32 + n / 8) + 8 * hh) = pk[mt];
                    }
                }
        }
        __syncthreads();

        // 2. h = [x | msg] . W1^T + b1; LayerNorm; GELU -> bf16 over [x | msg]
        {
            f32x16 acc[NT2][MT];
            zero(acc);
            FFN_T(3);
            if (!(MLG_FFN_PROBE & 8)) gemm_phase<NT2, MT, RING>(w.Wf1, 512, 32 * NT2 * wave, 8, 0, lds, acc);
            FFN_T(4);
    #pragma unroll
            for (int t = 0; t < NT2; ++t)
    #pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 b = *reinterpret_cast<const float4*>(s_bf1 + 32 * NT2 * wave + 32 * t + 8 * g + 4 * hh);
    #pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        acc[t][mt][4 * g] += b.x;
                        acc[t][mt][4 * g + 1] += b.y;
                        acc[t][mt][4 * g + 2] += b.z;
                        acc[t][mt][4 * g + 3] += b.w;
                    }
                }
            float mean[MT], rstd[MT];
    #pragma unroll
            for (int mt = 0; mt < MT; ++mt) { mean[mt] = 0.f; rstd[mt] = 1.f; }
    #pragma unroll
            for (int mt = 0; mt < MT && !relu && !(MLG_FFN_PROBE & 2); ++mt) {
                float sum = 0.f;
    #pragma unroll
                for (int t = 0; t < NT2; ++t)
    #pragma unroll
                    for (int i = 0; i < 16; ++i) sum += acc[t][mt][i];
                sum += __shfl_xor(sum, 32, 64);
                if (hh == 0) red[0][wave][32 * mt + col] = sum;
            }
            __syncthreads();  // also: every wave has finished reading [x | msg]
    #pragma unroll
            for (int mt = 0; mt < MT && !relu && !(MLG_FFN_PROBE & 2); ++mt) {
                float sum = 0.f;
    #pragma unroll
                for (int v = 0; v < NW; ++v) sum += red[0][v][32 * mt + col];
                mean[mt] = sum * (1.0f / 512.0f);
                float q = 0.f;
    #pragma unroll
                for (int t = 0; t < NT2; ++t)
    #pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const float d = acc[t][mt][i] - mean[mt];
                        q += d * d;
                    }
                q += __shfl_xor(q, 32, 64);
                if (hh == 0) red[1][wave][32 * mt + col] = q;
            }
            __syncthreads();
    #pragma unroll
            for (int mt = 0; mt < MT && !relu && !(MLG_FFN_PROBE & 2); ++mt) {
                float q = 0.f;
    #pragma unroll
                for (int v = 0; v < NW; ++v) q += red[1][v][32 * mt + col];
#if MLG_FFN_RSQ == 0
                rstd[mt] = rsqrtf(q * (1.0f / 512.0f) + 1e-5f);
#else
                // the bare v_rsq_f32: the argument is >= 1e-5, never in the range rsqrtf's
                // denormal fix-up handles, so the bits are the same (probe arm 2: followed by
                // 5 wait states before any consumer)
                rstd[mt] = __builtin_amdgcn_rsqf(q * (1.0f / 512.0f) + 1e-5f);
#if MLG_FFN_RSQ == 2
                asm volatile("s_nop 4" : "+v"(rstd[mt]));
#endif
#endif
            }
            FFN_T(5);
    #pragma unroll
            for (int t = 0; t < NT2; ++t)
    #pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int n = 32 * NT2 * wave + 32 * t + 8 * g + 4 * hh;
                    const float4 lg = *reinterpret_cast<const float4*>(s_lng + n);
                    const float4 lb = *reinterpret_cast<const float4*>(s_lnb + n);
                    uint2 pk[MT];
    #pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        const f32x16& a = acc[t][mt];
                        float y0, y1, y2, y3;
                        if (MLG_FFN_PROBE & 1) {
                            y0 = (a[4 * g] - mean[mt]) * rstd[mt] * lg.x + lb.x;
                            y1 = (a[4 * g + 1] - mean[mt]) * rstd[mt] * lg.y + lb.y;
                            y2 = (a[4 * g + 2] - mean[mt]) * rstd[mt] * lg.z + lb.z;
                            y3 = (a[4 * g + 3] - mean[mt]) * rstd[mt] * lg.w + lb.w;
                        } else if (relu) {
                            y0 = fmaxf(a[4 * g], 0.f);
                            y1 = fmaxf(a[4 * g + 1], 0.f);
                            y2 = fmaxf(a[4 * g + 2], 0.f);
                            y3 = fmaxf(a[4 * g + 3], 0.f);
                        } else {
                            const f32x2 u01 = gelu_poly2(f32x2{(a[4 * g] - mean[mt]) * rstd[mt] * lg.x + lb.x,
                                                               (a[4 * g + 1] - mean[mt]) * rstd[mt] * lg.y + lb.y});
                            const f32x2 u23 = gelu_poly2(f32x2{(a[4 * g + 2] - mean[mt]) * rstd[mt] * lg.z + lb.z,
                                                               (a[4 * g + 3] - mean[mt]) * rstd[mt] * lg.w + lb.w});
                            y0 = u01.x;
                            y1 = u01.y;
                            y2 = u23.x;
                            y3 = u23.y;
                        }
                        pk[mt] = make_uint2(pack_bf16x2(y0, y1), pack_bf16x2(y2, y3));
                    }
                    if constexpr (MLG_FFN_STAGE_W && MT == 2) {
                        cat_pair_write(lds, n / 8, pk[0], pk[MT - 1]);
                    } else {
    #pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
                            *reinterpret_cast<uint2*>(lds + cat_off(32 * mt + col, n / 8) + 8 * hh) = pk[mt];
                    }
                }
        }
        __syncthreads();

        // 3. x += GELU(..) . W2^T + b2 (f32); bf16 copy of x for the next projections.
        //    y = acc + b2 is staged in LDS ([64][256] f32 over the dead GELU tile, 16-B chunk
        //    c of row r at c ^ (r & 15)), then each wave streams whole rows: 64 lanes x 16 B =
        //    one 1-KiB f32 row of x read, updated and written, its 512-B bf16 copy written --
        //    full-line HBM traffic instead of 16-B pieces of 32 rows per instruction.
        {
            // the residual rows this wave updates below, fetched now so their HBM latency
            // hides under the ffn2 GEMM (rows past M clamped, never stored)
            float4 xr[R / NW];
    #pragma unroll
            for (int i = 0; i < R / NW; ++i)
                xr[i] = stream_ld(reinterpret_cast<const float4*>(X + (size_t)min(m0 + wave * (R / NW) + i, M - 1) * 256) + lane);
            __builtin_amdgcn_sched_barrier(0);
            f32x16 acc[NT1][MT];
            zero(acc);
            FFN_T(6);
            if (!(MLG_FFN_PROBE & 16)) gemm_phase<NT1, MT, RING1>(w.Wf2, 256, 32 * NT1 * wave, 8, 0, lds, acc);
            FFN_T(7);
#if MLG_FFN_XR_WAIT
            __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0): the residual rows xr have landed
#endif
            __syncthreads();  // every wave has read the GELU output
    #pragma unroll
            for (int t = 0; t < NT1; ++t)
    #pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int n = 32 * NT1 * wave + 32 * t + 8 * g + 4 * hh;
                    const float4 b = *reinterpret_cast<const float4*>(s_bf2 + n);
    #pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        const int r = 32 * mt + col;
                        const f32x16& a = acc[t][mt];
                        *reinterpret_cast<float4*>(lds + r * 1024 + (((n >> 2) ^ (r & 15)) << 4)) =
                            make_float4(a[4 * g] + b.x, a[4 * g + 1] + b.y, a[4 * g + 2] + b.z, a[4 * g + 3] + b.w);
                    }
                }
            __syncthreads();
            FFN_T(8);
            // Heads (cf.wm != nullptr): each lane keeps its 4-column partial dot of each of
            // the wave's 16 rows; one reduce-scatter over the 64 lanes (8 + 4 + 2 + 1 + 1 + 1
            // shuffles per head instead of 16 x 6) leaves every 4-lane group with one row's sum.
            const bool heads = cf.wm != nullptr, conf = cf.wc != nullptr;
            float4 wm4 = make_float4(0.f, 0.f, 0.f, 0.f), wc4 = wm4;
            if (heads) wm4 = *reinterpret_cast<const float4*>(cf.wm + 4 * lane);
            if (conf) wc4 = *reinterpret_cast<const float4*>(cf.wc + 4 * lane);
            float pz[R / NW], pa[R / NW];
    #pragma unroll
            for (int i = 0; i < R / NW; ++i) {
                const int r = wave * (R / NW) + i, m = m0 + r;
                pz[i] = pa[i] = 0.f;
                if (m >= M || (MLG_FFN_PROBE & 32)) continue;  // wave-uniform
                const float4 y = *reinterpret_cast<const float4*>(lds + r * 1024 + ((lane ^ (r & 15)) << 4));
                float4* px = reinterpret_cast<float4*>(X + (size_t)m * 256) + lane;
                float4 x = xr[i];
                if constexpr (LOFTR) {  // norm2 over the row (one wave = one 256-wide row)
                    const float mean = wave_sum(y.x + y.y + y.z + y.w) * (1.0f / 256.0f);
                    const float d0 = y.x - mean, d1 = y.y - mean, d2 = y.z - mean, d3 = y.w - mean;
                    const float q = wave_sum(fmaf(d3, d3, fmaf(d2, d2, fmaf(d1, d1, d0 * d0))));
                    const float rstd = 1.0f / sqrtf(q * (1.0f / 256.0f) + 1e-5f);
                    const float4 lg = *reinterpret_cast<const float4*>(s_lng + 256 + 4 * lane);
                    const float4 lb = *reinterpret_cast<const float4*>(s_lnb + 256 + 4 * lane);
                    x.x += d0 * rstd * lg.x + lb.x;
                    x.y += d1 * rstd * lg.y + lb.y;
                    x.z += d2 * rstd * lg.z + lb.z;
                    x.w += d3 * rstd * lg.w + lb.w;
                } else {
                    x.x += y.x;
                    x.y += y.y;
                    x.z += y.z;
                    x.w += y.w;
                }
                stream_st(px, x);
                *reinterpret_cast<uint2*>(xcopy + (size_t)m * ldc + 4 * lane) =
                    make_uint2(pack_bf16x2(x.x, x.y), pack_bf16x2(x.z, x.w));
                if (heads) pz[i] = x.x * wm4.x + x.y * wm4.y + x.z * wm4.z + x.w * wm4.w;
                if (conf) pa[i] = x.x * wc4.x + x.y * wc4.y + x.z * wc4.z + x.w * wc4.w;
            }
            if (heads) {
                // reduce-scatter: after the step over lane bit b the lane keeps the half of its
                // rows selected by that bit; rows end up as row = 8 b5 + 4 b4 + 2 b3 + b2
    #pragma unroll
                for (int half = 8, bit = 32; half >= 1; half >>= 1, bit >>= 1) {
                    const bool up = (lane & bit) != 0;
    #pragma unroll
                    for (int j = 0; j < half; ++j) {
                        const float kz = up ? pz[half + j] : pz[j], sz = up ? pz[j] : pz[half + j];
                        pz[j] = kz + __shfl_xor(sz, bit, 64);
                        if (conf) {
                            const float ka = up ? pa[half + j] : pa[j], sa = up ? pa[j] : pa[half + j];
                            pa[j] = ka + __shfl_xor(sa, bit, 64);
                        }
                    }
                }
                float z = pz[0], a = pa[0];
                z += __shfl_xor(z, 2, 64);
                z += __shfl_xor(z, 1, 64);
                if (conf) {
                    a += __shfl_xor(a, 2, 64);
                    a += __shfl_xor(a, 1, 64);
                }
                const int r = wave * (R / NW) + (lane >> 2), m = m0 + r;
                if ((lane & 3) == 0 && m < M) {  // one writer per row (k_lg_conf semantics)
                    z += cf.bm[0];
                    if (cf.rowseg[m] < 0) {
                        if (conf) cf.flags[m] = 0;
                    } else {
                        cf.lz[m] = logsigmoid_f(z);
                        if (conf) {
                            const float c = sigmoid_f(a + cf.bc[0]);
                            const bool keep = sigmoid_f(z) > 1.f - cf.width || c <= cf.thr;
                            cf.flags[m] = (uint8_t)((c < cf.thr) | (keep << 1));
                        }
                    }
                }
            }
        }
#if MLG_FFN_TRACE
        FFN_T(9);
        if (threadIdx.x == 0 && blockIdx.x < FFN_TRACE_WGS) {
            unsigned long long* o = g_ffn_trace + (size_t)blockIdx.x * FFN_TRACE_W;
    #pragma unroll
            for (int i = 0; i < 10; ++i) o[i] = tt[i];
            o[10] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID
            o[11] = (unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
        }
#endif
        if (!PERSIST) break;  // one tile per workgroup: no loop, no state carried across tiles
        __syncthreads();  // the next tile overwrites the LDS image
    }
}

[[maybe_unused]] int ffn_num_cus() {
    static const int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1)
            return 256;
        return c;
    }();
    return n;
}

}  // namespace

// copies the phase trace of a MLG_FFN_TRACE build ([FFN_TRACE_WGS][12] u64); -1 otherwise
extern "C" int mlg_dbg_ffn_trace(void* host, size_t bytes) {
#if MLG_FFN_TRACE
    const size_t n = std::min(bytes, sizeof(g_ffn_trace));
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ffn_trace), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : MLG_EHIP;
#else
    (void)host;
    (void)bytes;
    return MLG_EINVAL;
#endif
}

int mlg_lg_ffn(const bf16_t* ctx, float* X, bf16_t* xcopy, int ldc, int M, const mlg_lg_block_i& w, hipStream_t s,
               const mlg_lg_conf_i* conf, int relu) {
    if (M <= 0) return MLG_OK;
    if (ldc < 256 || (ldc % 8) || relu < 0 || relu > 2) return MLG_EINVAL;
    if (relu == 2 && (MLG_FFN_ROWS != 64 || MLG_FFN_GRID > 0)) return MLG_EINVAL;  // LoFTR form: default launch only
    mlg_lg_conf_i cf{};
    if (conf) cf = *conf;
#if MLG_FFN_ROWS == 128
    if (relu)
        hipLaunchKernelGGL((k_lg_ffn<false, 128, 8, false, true>), dim3((unsigned)((M + 127) / 128)), dim3(512), 0, s,
                           ctx, X, xcopy, ldc, M, w, cf);
    else
        hipLaunchKernelGGL((k_lg_ffn<false, 128, 8>), dim3((unsigned)((M + 127) / 128)), dim3(512), 0, s, ctx, X, xcopy,
                           ldc, M, w, cf);
#elif MLG_FFN_GRID > 0
    const long ntiles = (M + 63) / 64;
    const long grid = std::min<long>(ntiles, (long)MLG_FFN_GRID * ffn_num_cus());
    if (relu)
        hipLaunchKernelGGL((k_lg_ffn<true, 64, 4, false, true>), dim3((unsigned)grid), dim3(256), 0, s, ctx, X, xcopy,
                           ldc, M, w, cf);
    else
        hipLaunchKernelGGL((k_lg_ffn<true, 64, 4>), dim3((unsigned)grid), dim3(256), 0, s, ctx, X, xcopy, ldc, M, w, cf);
#else
    const long ntiles = (M + 63) / 64;
    if (relu == 2)
        hipLaunchKernelGGL((k_lg_ffn<false, 64, 4, true>), dim3((unsigned)ntiles), dim3(256), 0, s, ctx, X, xcopy, ldc,
                           M, w, cf);
    else if (relu == 1)
        hipLaunchKernelGGL((k_lg_ffn<false, 64, 4, false, true>), dim3((unsigned)ntiles), dim3(256), 0, s, ctx, X, xcopy,
                           ldc, M, w, cf);
    else
        hipLaunchKernelGGL((k_lg_ffn<false, 64, 4>), dim3((unsigned)ntiles), dim3(256), 0, s, ctx, X, xcopy, ldc, M, w,
                           cf);
#endif
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}
