// Fused multi-head attention on gfx950: one software-pipelined tile (k_attention_varlen)
// serves the ViT-B/14 (12 heads x 64, T = 530 tokens at 322^2; hub Attention.forward
//   O[b, t, h*64 + d] = softmax_k( q_t . k_k / 8 ) . v_k )
// and LightGlue's ragged self / cross attention (4 heads x 64).
//
// Scores are computed transposed, S^T = K . Q^T, with v_mfma_f32_32x32x16_bf16 so
// that a lane owns one query column: the softmax row statistics are lane-local plus
// one cross-half exchange, and the S^T accumulator feeds the next MFMA directly as
// its B operand (O^T = V^T . P^T) with no LDS round trip.  O^T keeps the query on
// the lane too, so the online-softmax rescale is lane-local.
//
// Layouts (ViT: written by the QKV GEMM epilogue, gemm_bf16.hip EpiQKV; one task per
// image over the segment b * Tpad of every head):
//   Q, K : bf16 [heads][Npad][64];   Vt : bf16 [heads][Npad / 64][64 d][64 keys]
//   V^T columns of keys >= T must be finite (zeroed per forward); keys >= T are masked.
// Output O: bf16 rows of ldo elements, head h at column h * 64.
#include "common.h"
#include "kernels.h"

namespace {

// Phase timestamps (probe builds, MLG_ATT_TRACE=1; 0 in the product): per LightGlue
// workgroup s_memtime at entry, after the prologue barrier, after the stage loop and at
// the end, with HW_ID / XCC_ID (mlg_dbg_att_trace, tools/attn_trace.py)
#ifndef MLG_ATT_TRACE
#define MLG_ATT_TRACE 0
#endif
[[maybe_unused]] constexpr int ATT_TRACE_WGS = 1 << 16;
#if MLG_ATT_TRACE
__device__ unsigned long long g_att_trace[ATT_TRACE_WGS * 8];
#define ATT_T(i) att_tt[i] = __builtin_amdgcn_s_memtime()
#else
#define ATT_T(i) (void)0
#endif
// Staging writes by the calibrated LDS write rule (writes retire 128 B per cycle in lane
// order -- b64: 16 lanes, b128: 8 lanes -- and conflict unless those lanes hit distinct
// banks modulo 128 B; profiles/r05x_lds_calibration.txt): the K / V staging lanes take
// rows (r, r + 2) per 16-lane group instead of (r, r + 1), whose V^T granule swizzles
// differ in bit 0, so the two rows' b64 writes fill disjoint halves of the 128-B window;
// the O epilogue pairs lanes l / l + 32 (v_permlane32_swap) into whole-chunk b128 writes.
// 0: the round-4 staging (A/B only).
#ifndef MLG_ATT_STAGE_W
#define MLG_ATT_STAGE_W 1
#endif
constexpr int KB = 64;                 // keys per block
constexpr int KTILE_BYTES = KB * 128;  // 64 rows x 64 bf16
constexpr int VTILE_BYTES = 64 * KB * 2;
// SPLIT: the lo V^T tile of a ring slot starts 8 B past the hi tile's end.  At exactly
// VTILE_BYTES (a multiple of 512 B) hipcc fused each hi / lo pair of fragment reads into
// one ds_read2st64_b64, which banks modulo 32 dwords and 2-way conflicts (the split ViT
// tile's PMC conflict share 0.67-0.76, round 6); 8200 B apart no ds_read2 form applies, and a
// uniform 8-B shift keeps the image's bank pattern.
constexpr int VLO = VTILE_BYTES + 8;

__device__ __forceinline__ int k_off(int key, int chunk) {  // K image [key][d], 16-B chunks
    return key * 128 + ((chunk ^ ((key >> 1) & 7)) << 4);
}
// V^T image [d][key], 8-B granules.  The (d >> 5) term makes the d and d + 32 rows of
// one lane non-constant apart, so hipcc cannot fuse the two ds_read_b64 into a
// ds_read2st64_b64 (which banks mod 32 dwords and would 2-way conflict).
__device__ __forceinline__ int v_off(int d, int gran) {
    return d * 128 + ((gran ^ (((d >> 1) ^ (d >> 5)) & 15)) << 3);
}

// Software-pipelined wide tile for the ragged (LightGlue) path: one workgroup = 4 waves
// = 256 query rows of one (task, head), one wave per SIMD, each wave 64 queries as two
// 32-column MFMA tiles.  The softmax runs over 32-key half-blocks: while the VALU
// exponentiates half-block h (scores computed one step earlier) and P_h V_h runs, the
// MFMA pipe computes the scores of half-block h + 1, so every MFMA gap has independent
// VALU work (a one-phase tile leaves the VALU idle during QK^T and the MFMA pipe idle
// during the max / exp chain: 865 vs 936 TFLOP/s on bench.py's LightGlue stage).  Two 32-key score sets (64 VGPRs) are live.
// VALU per score, the bound of a d = 64 attention: no key mask except in the last stage;
// (written as packed f32 -- f32x2 fma / adds, round 4 -- hipcc allocates the pairs out of the
// MFMA accumulators with 418 extra v_mov_b64 and 238 v_accvgpr_read per kernel: 3882 vs
// 3460 VALU instructions, so the scalar forms stay)
// exponent as one fma + one v_exp (log2 domain, 1/8 folded into the constant); row sums
// as f32 adds per lane half (a 16x16x32 ones-MFMA for them measured slower); the running
// max moves lazily -- P and the O / l
// accumulators are rescaled only when some lane's max grows by more than 2^8, so
// P <= 256 (exact softmax either way: numerator and denominator share the stale max).
// Softmax order is the textbook one: a half-block's max and the lazy rescale decision
// precede its exponentials, and all earlier P V MFMAs have been
// issued by then.
// LDS, per 64-key stage: K ring of 3 (the current stage's K is still read for its second
// half while K_{j+1} is read and K_{j+2} lands), V ring of 3 (slot j % 3 like K: the stage
// loop is unrolled by 3 so every ring address is a constant); global loads issued at the
// top of a stage land in LDS at its end, one barrier per stage.
__device__ __forceinline__ float swap_sum(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Row max of each query tile's 16 scores, merged with the other lane half (permlane32
// swap) -- ONE asm statement: hipcc pads every inline-asm statement with an s_nop (it
// cannot see inside) and puts a NaN-canonicalising v_max_f32 in front of every fmaxf
// operand it did not produce, so per-instruction statements or fmaxf on the swap results
// cost as much again as the maxima.  The two chains interleave; `s_nop 1`: the VALU-write
// -> permlane32_swap-read wait states.  Scores are finite or -inf.
// The scores are MFMA results read by the asm: an XDL write -> VALU read needs 12 wait
// states after an 8-pass v_mfma_f32_32x32x16_bf16, and hipcc inserts none for a consumer
// inside an asm string.  Wherever the scheduler put the producing MFMAs close to this
// read, the max came from accumulators not yet written, on some waves, under load: up to
// ~0.1 % of output rows differed run to run (tools/attn_det_probe.py, 0 with the pad;
// the pad costs ~0.8 % of the tile's time).  The pad is tied to the inputs so it sits
// between their producers and this read.
__device__ __forceinline__ void block_max2(f32x16 (&v)[2], float (&m)[2]) {
    float a, b, t0, t1;
    asm volatile("s_nop 11" : "+v"(v[0][15]), "+v"(v[1][15]));
    asm("v_max3_f32 %0, %4, %5, %6\n\t"
        "v_max3_f32 %1, %20, %21, %22\n\t"
        "v_max3_f32 %0, %0, %7, %8\n\t"
        "v_max3_f32 %1, %1, %23, %24\n\t"
        "v_max3_f32 %0, %0, %9, %10\n\t"
        "v_max3_f32 %1, %1, %25, %26\n\t"
        "v_max3_f32 %0, %0, %11, %12\n\t"
        "v_max3_f32 %1, %1, %27, %28\n\t"
        "v_max3_f32 %0, %0, %13, %14\n\t"
        "v_max3_f32 %1, %1, %29, %30\n\t"
        "v_max3_f32 %0, %0, %15, %16\n\t"
        "v_max3_f32 %1, %1, %31, %32\n\t"
        "v_max3_f32 %0, %0, %17, %18\n\t"
        "v_max3_f32 %1, %1, %33, %34\n\t"
        "v_max3_f32 %0, %0, %19, %19\n\t"
        "v_max3_f32 %1, %1, %35, %35\n\t"
        "v_mov_b32 %2, %0\n\t"
        "v_mov_b32 %3, %1\n\t"
        "s_nop 1\n\t"
        "v_permlane32_swap_b32 %0, %2\n\t"
        "v_permlane32_swap_b32 %1, %3\n\t"
        "v_max_f32 %0, %0, %2\n\t"
        "v_max_f32 %1, %1, %3"
        : "=&v"(a), "=&v"(b), "=&v"(t0), "=&v"(t1)
        : "v"(v[0][0]), "v"(v[0][1]), "v"(v[0][2]), "v"(v[0][3]), "v"(v[0][4]), "v"(v[0][5]), "v"(v[0][6]),
          "v"(v[0][7]), "v"(v[0][8]), "v"(v[0][9]), "v"(v[0][10]), "v"(v[0][11]), "v"(v[0][12]), "v"(v[0][13]),
          "v"(v[0][14]), "v"(v[0][15]),
          "v"(v[1][0]), "v"(v[1][1]), "v"(v[1][2]), "v"(v[1][3]), "v"(v[1][4]), "v"(v[1][5]), "v"(v[1][6]),
          "v"(v[1][7]), "v"(v[1][8]), "v"(v[1][9]), "v"(v[1][10]), "v"(v[1][11]), "v"(v[1][12]), "v"(v[1][13]),
          "v"(v[1][14]), "v"(v[1][15]));
    m[0] = a;
    m[1] = b;
}

// One query tile (the 8-wave form, 32 queries per wave): the same chain, one column.
__device__ __forceinline__ void block_max1(f32x16 (&v)[1], float (&m)[1]) {
    float a, t0;
    asm volatile("s_nop 11" : "+v"(v[0][15]));
    asm("v_max3_f32 %0, %2, %3, %4\n\t"
        "v_max3_f32 %0, %0, %5, %6\n\t"
        "v_max3_f32 %0, %0, %7, %8\n\t"
        "v_max3_f32 %0, %0, %9, %10\n\t"
        "v_max3_f32 %0, %0, %11, %12\n\t"
        "v_max3_f32 %0, %0, %13, %14\n\t"
        "v_max3_f32 %0, %0, %15, %16\n\t"
        "v_max3_f32 %0, %0, %17, %17\n\t"
        "v_mov_b32 %1, %0\n\t"
        "s_nop 1\n\t"
        "v_permlane32_swap_b32 %0, %1\n\t"
        "v_max_f32 %0, %0, %1"
        : "=&v"(a), "=&v"(t0)
        : "v"(v[0][0]), "v"(v[0][1]), "v"(v[0][2]), "v"(v[0][3]), "v"(v[0][4]), "v"(v[0][5]), "v"(v[0][6]),
          "v"(v[0][7]), "v"(v[0][8]), "v"(v[0][9]), "v"(v[0][10]), "v"(v[0][11]), "v"(v[0][12]), "v"(v[0][13]),
          "v"(v[0][14]), "v"(v[0][15]));
    m[0] = a;
}

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

// SPLIT (the ViT's MLG_VIT_SPLIT forward): Q / K / V^T each come as a hi plane and a lo
// plane (x = hi + lo, lo_off elements apart); a K / V ring slot holds the hi tile and then
// the lo tile; every product is hi*hi + lo*hi + hi*lo (three MFMAs into one accumulator)
// and P is split in registers after the exponential.
template <bool SPLIT>
struct Slots {
    static constexpr int K = SPLIT ? 2 * KTILE_BYTES : KTILE_BYTES;
    static constexpr int V = SPLIT ? 2 * VTILE_BYTES + 16 : VTILE_BYTES;  // + 16: slots stay 16-B aligned
};

struct PipeCtx {
    const bf16_t* Kh;
    const bf16_t* Vh;
    const bf16_t* Kl;  // lo planes (SPLIT only)
    const bf16_t* Vl;
    char* smem;
    int T, nkb, gk_off, gv_off;
    int sk0, sk1, sv0a, sv0b, sv1a, sv1b;
    int koff[4];     // K fragment offset per 16-key step (chunk XOR depends on it only)
    int voff[2][2][4];  // V^T fragment offsets [half][st][dt * 2 + lo/hi]
};

// S^T of one 32-key half-block (kt) of the K tile at kb: [qt] tiles.
// HAZARD PAD CONTRACT (block_max2's `s_nop 11`): the scores read by the asm row max must
// come from v_mfma_f32_32x32x16_bf16 -- an 8-pass XDL op on gfx950, whose result needs 12
// wait states before a VALU read -- each writing the WHOLE f32x16 accumulator (the pad is
// tied to element [15]).  Changing this MFMA's shape (e.g. 16x16x32, 4 passes) or
// splitting the accumulator requires re-deriving the pad; tests/test_kernels_gpu.py's
// attention bit-identity test is the run-time guard.
template <bool SPLIT, int QT>
__device__ __forceinline__ void qk_half(const char* kb, const PipeCtx& c, const bf16x8 (&qf)[QT][4],
                                        const bf16x8 (&qfl)[QT][4], int kt, f32x16 (&s)[QT]) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) s[qt][i] = 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + kt * 4096 + c.koff[st]);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) s[qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[qt][st], s[qt], 0, 0, 0);
        if (SPLIT) {
            const bf16x8 kl = *reinterpret_cast<const bf16x8*>(kb + KTILE_BYTES + kt * 4096 + c.koff[st]);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                s[qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qf[qt][st], s[qt], 0, 0, 0);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                s[qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qfl[qt][st], s[qt], 0, 0, 0);
        }
    }
}

template <int QT>
__device__ __forceinline__ void block_max(f32x16 (&v)[QT], float (&m)[QT]) {
    if constexpr (QT == 2) block_max2(v, m);
    else block_max1(v, m);
}

// half-step H of stage j: consume `cur` (keys 64 j + 32 H ..), produce `nxt`.  kcur /
// knext: K ring slots of stages j / j + 1; kw: slot for K_{j+2}.
// QT query tiles of 32 per wave (2: the 4-wave form, 64 queries per wave; 1: the 8-wave
// form, 32 per wave -- two waves per SIMD where the tile's registers allow only one wave
// of the 4-wave form); SP = K / V staging rows per thread per plane (2 for 256 threads, 1
// for 512)
template <int H, bool LASTSTAGE, int R, bool SPLIT, int QT>
__device__ __forceinline__ void pipe_half(int j, f32x16 (&cur)[QT], f32x16 (&nxt)[QT], const PipeCtx& c,
                                          const bf16x8 (&qf)[QT][4], const bf16x8 (&qfl)[QT][4], f32x16 (&o)[QT][2],
                                          float (&mrun)[QT], float (&lsum)[QT][2], uint4 (&stage)[4 * QT],
                                          int rr = 0, bool busy = true) {
    constexpr int KS = Slots<SPLIT>::K, VS = Slots<SPLIT>::V;
    constexpr int SP = QT;  // 256 threads (QT 2): rows srow and srow + 32; 512 threads: row srow
    // ring slots are compile-time constants (stage j uses K slot j % 3 = R, V slot R), so
    // every LDS fragment address is a lane offset plus an immediate; R < 0: slot rr at run
    // time (the last stage only)
    const int rs = R >= 0 ? R : rr;
    const int kcur = rs * KS, knext = ((rs + 1) % 3) * KS, kw = ((rs + 2) % 3) * KS;
    constexpr float C = 0.125f * 1.4426950408889634f;  // 1/sqrt(64) * log2(e)
    const int hh = (threadIdx.x & 63) >> 5;
    if (!LASTSTAGE && H == 0) {  // K_{j+2} (clamped), V_{j+1} -> registers, into LDS at the stage end
        const bf16_t* pk = c.Kh + (size_t)min(j + 2, c.nkb - 1) * (KB * 64) + c.gk_off;
        stage[0] = *reinterpret_cast<const uint4*>(pk);
        if (SP == 2) stage[1] = *reinterpret_cast<const uint4*>(pk + 32 * 64);
        const bf16_t* pv = c.Vh + (size_t)(j + 1) * 4096 + c.gv_off;
        stage[SP] = *reinterpret_cast<const uint4*>(pv);
        if (SP == 2) stage[3] = *reinterpret_cast<const uint4*>(pv + 32 * 64);
        if (SPLIT) {
            const bf16_t* pkl = c.Kl + (size_t)min(j + 2, c.nkb - 1) * (KB * 64) + c.gk_off;
            stage[2 * SP] = *reinterpret_cast<const uint4*>(pkl);
            if (SP == 2) stage[5] = *reinterpret_cast<const uint4*>(pkl + 32 * 64);
            const bf16_t* pvl = c.Vl + (size_t)(j + 1) * 4096 + c.gv_off;
            stage[3 * SP] = *reinterpret_cast<const uint4*>(pvl);
            if (SP == 2) stage[7] = *reinterpret_cast<const uint4*>(pvl + 32 * 64);
        }
    }
    // 8-wave split form: a wave whose 32 queries all lie past the segment (the ViT's third
    // query block: 18 of 256 rows live) only stages K / V and joins the barriers
    const bool run = !(SPLIT && QT == 1) || busy;
    if (run) {
    if (LASTSTAGE && (c.T & (KB - 1))) {  // partial last stage: mask keys >= T
        const int key0 = j * KB + H * 32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int key = key0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (key >= c.T)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) cur[qt][r] = -INFINITY;
        }
    }
    float mnew[QT];
    bool grow = false;
    float bm[QT];
    block_max<QT>(cur, bm);  // both lane halves
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        mnew[qt] = fmaxf(mrun[qt], bm[qt]);
        grow |= (mnew[qt] - mrun[qt]) * C > 8.0f;
    }
    if (__any(grow)) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const float alpha = __builtin_amdgcn_exp2f((mrun[qt] - mnew[qt]) * C);
            lsum[qt][0] *= alpha;
            lsum[qt][1] *= alpha;
#pragma unroll
            for (int i = 0; i < 16; ++i) { o[qt][0][i] *= alpha; o[qt][1][i] *= alpha; }
            mrun[qt] = mnew[qt];
        }
    }
    float mc[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) mc[qt] = mrun[qt] * C;
    // next half-block's scores on the MFMA pipe
    const char* kring = c.smem;
    if (!(LASTSTAGE && H == 1)) qk_half<SPLIT, QT>(kring + (H == 0 ? kcur : knext), c, qf, qfl, H ^ 1, nxt);
    // P of this half-block [st][qt]: keys 16 st + 8 hh .. + 7, then O^T += V^T . P^T
    const char* vb = c.smem + 3 * KS + rs * VS;
    bf16x8 pf[2][QT], pfl[2][QT];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            u32x4 w, wl;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const float p0 = __builtin_amdgcn_exp2f(fmaf(cur[qt][8 * st + 2 * jj], C, -mc[qt]));
                const float p1 = __builtin_amdgcn_exp2f(fmaf(cur[qt][8 * st + 2 * jj + 1], C, -mc[qt]));
                lsum[qt][0] += p0;
                lsum[qt][1] += p1;
                w[jj] = pack_bf16x2(p0, p1);
                if (SPLIT)
                    wl[jj] = pack_bf16x2(p0 - __uint_as_float(w[jj] << 16), p1 - __uint_as_float(w[jj] & 0xffff0000u));
            }
            pf[st][qt] = __builtin_bit_cast(bf16x8, w);
            if (SPLIT) pfl[st][qt] = __builtin_bit_cast(bf16x8, wl);
        }
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const s16x4 lo = *reinterpret_cast<const s16x4*>(vb + c.voff[H][st][2 * dt]);
            const s16x4 hi = *reinterpret_cast<const s16x4*>(vb + c.voff[H][st][2 * dt + 1]);
            const bf16x8 vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
                o[qt][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[st][qt], o[qt][dt], 0, 0, 0);
            if (SPLIT) {
                const s16x4 llo = *reinterpret_cast<const s16x4*>(vb + VLO + c.voff[H][st][2 * dt]);
                const s16x4 lhi = *reinterpret_cast<const s16x4*>(vb + VLO + c.voff[H][st][2 * dt + 1]);
                const bf16x8 vl = __builtin_shufflevector(llo, lhi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
                    o[qt][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl, pf[st][qt], o[qt][dt], 0, 0, 0);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
                    o[qt][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pfl[st][qt], o[qt][dt], 0, 0, 0);
            }
        }
    }
    }  // run
    if (!LASTSTAGE && H == 1) {
        char* kwp = c.smem + kw;
        char* vw = c.smem + 3 * KS + ((rs + 1) % 3) * VS;
        *reinterpret_cast<uint4*>(kwp + c.sk0) = stage[0];
        if (SP == 2) *reinterpret_cast<uint4*>(kwp + c.sk1) = stage[1];
        *reinterpret_cast<uint2*>(vw + c.sv0a) = make_uint2(stage[SP].x, stage[SP].y);
        *reinterpret_cast<uint2*>(vw + c.sv0b) = make_uint2(stage[SP].z, stage[SP].w);
        if (SP == 2) {
            *reinterpret_cast<uint2*>(vw + c.sv1a) = make_uint2(stage[3].x, stage[3].y);
            *reinterpret_cast<uint2*>(vw + c.sv1b) = make_uint2(stage[3].z, stage[3].w);
        }
        if (SPLIT) {
            *reinterpret_cast<uint4*>(kwp + KTILE_BYTES + c.sk0) = stage[2 * SP];
            if (SP == 2) *reinterpret_cast<uint4*>(kwp + KTILE_BYTES + c.sk1) = stage[5];
            char* vl = vw + VLO;
            *reinterpret_cast<uint2*>(vl + c.sv0a) = make_uint2(stage[3 * SP].x, stage[3 * SP].y);
            *reinterpret_cast<uint2*>(vl + c.sv0b) = make_uint2(stage[3 * SP].z, stage[3 * SP].w);
            if (SP == 2) {
                *reinterpret_cast<uint2*>(vl + c.sv1a) = make_uint2(stage[7].x, stage[7].y);
                *reinterpret_cast<uint2*>(vl + c.sv1b) = make_uint2(stage[7].z, stage[7].w);
            }
        }
        __syncthreads();
    }
}

template <bool SPLIT, int NW = 4>
__device__ __forceinline__ void attention_tile_pipe(unsigned long long* att_tt, char* smem, const bf16_t* __restrict__ Qh,
                                                    const bf16_t* __restrict__ Kh, const bf16_t* __restrict__ Vh,
                                                    int T, int nq, int qmax, int qblock, bf16_t* __restrict__ orow,
                                                    int ldo, size_t lo_off, int lo_col) {
    constexpr int KS = Slots<SPLIT>::K;
    constexpr int QT = NW == 4 ? 2 : 1;  // query tiles of 32 per wave: 256 queries per workgroup
    constexpr int SP = QT;               // K / V staging rows per thread per plane
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5, col = lane & 31;
    const int qbase = qblock * 256 + wave * 32 * QT;
    bf16x8 qf[QT][4], qfl[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int qld = min(qbase + qt * 32 + col, qmax - 1);
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            qf[qt][st] = *reinterpret_cast<const bf16x8*>(Qh + (size_t)qld * 64 + st * 16 + hh * 8);
            if (SPLIT) qfl[qt][st] = *reinterpret_cast<const bf16x8*>(Qh + lo_off + (size_t)qld * 64 + st * 16 + hh * 8);
        }
    }
    PipeCtx c;
    c.Kh = Kh;
    c.Vh = Vh;
    c.Kl = Kh + lo_off;
    c.Vl = Vh + lo_off;
    c.smem = smem;
    c.T = T;
    c.nkb = (T + KB - 1) / KB;
    // rows srow (+ 32 when 256 threads) of each 64-row tile; MLG_ATT_STAGE_W: 16-lane group k
    // stages rows b, b + 2 with b = 4 (k >> 1) + (k & 1) (a bijection onto the same rows)
    const int sg = tid >> 4;
    const int srow = MLG_ATT_STAGE_W ? 4 * (sg >> 1) + (sg & 1) + 2 * ((tid >> 3) & 1) : tid >> 3, sch = tid & 7;
    c.gk_off = srow * 64 + sch * 8;
    c.gv_off = srow * 64 + sch * 8;
    c.sk0 = k_off(srow, sch);
    c.sk1 = k_off(srow + 32, sch);
    c.sv0a = v_off(srow, 2 * sch);
    c.sv0b = v_off(srow, 2 * sch + 1);
    c.sv1a = v_off(srow + 32, 2 * sch);
    c.sv1b = v_off(srow + 32, 2 * sch + 1);
#pragma unroll
    for (int st = 0; st < 4; ++st) c.koff[st] = k_off(col, 2 * st + hh);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {  // 8-B granule of keys 32 h + 16 st + 4 hh (+ 8)
                c.voff[h][st][2 * dt] = v_off(dt * 32 + col, h * 8 + st * 4 + hh);
                c.voff[h][st][2 * dt + 1] = v_off(dt * 32 + col, h * 8 + st * 4 + hh + 2);
            }
    {
        // (rows srow + 32 only with 256 threads; the same statement order as the 4-wave tile)
        const uint4 k0 = *reinterpret_cast<const uint4*>(Kh + c.gk_off);
        const uint4 k1 = SP == 2 ? *reinterpret_cast<const uint4*>(Kh + c.gk_off + 32 * 64) : k0;
        const uint4 v0 = *reinterpret_cast<const uint4*>(Vh + c.gv_off);
        const uint4 v1 = SP == 2 ? *reinterpret_cast<const uint4*>(Vh + c.gv_off + 32 * 64) : v0;
        const bf16_t* pk = Kh + (size_t)min(1, c.nkb - 1) * (KB * 64) + c.gk_off;
        const uint4 k2 = *reinterpret_cast<const uint4*>(pk);
        const uint4 k3 = SP == 2 ? *reinterpret_cast<const uint4*>(pk + 32 * 64) : k2;
        *reinterpret_cast<uint4*>(smem + c.sk0) = k0;
        if (SP == 2) *reinterpret_cast<uint4*>(smem + c.sk1) = k1;
        *reinterpret_cast<uint4*>(smem + KS + c.sk0) = k2;
        if (SP == 2) *reinterpret_cast<uint4*>(smem + KS + c.sk1) = k3;
        char* vw = smem + 3 * KS;
        *reinterpret_cast<uint2*>(vw + c.sv0a) = make_uint2(v0.x, v0.y);
        *reinterpret_cast<uint2*>(vw + c.sv0b) = make_uint2(v0.z, v0.w);
        if (SP == 2) {
            *reinterpret_cast<uint2*>(vw + c.sv1a) = make_uint2(v1.x, v1.y);
            *reinterpret_cast<uint2*>(vw + c.sv1b) = make_uint2(v1.z, v1.w);
        }
        if (SPLIT) {
            const bf16_t* Kl = c.Kl;
            const bf16_t* Vl = c.Vl;
            const uint4 l0 = *reinterpret_cast<const uint4*>(Kl + c.gk_off);
            const uint4 l1 = SP == 2 ? *reinterpret_cast<const uint4*>(Kl + c.gk_off + 32 * 64) : l0;
            const uint4 w0 = *reinterpret_cast<const uint4*>(Vl + c.gv_off);
            const uint4 w1 = SP == 2 ? *reinterpret_cast<const uint4*>(Vl + c.gv_off + 32 * 64) : w0;
            const bf16_t* pl = Kl + (size_t)min(1, c.nkb - 1) * (KB * 64) + c.gk_off;
            const uint4 l2 = *reinterpret_cast<const uint4*>(pl);
            const uint4 l3 = SP == 2 ? *reinterpret_cast<const uint4*>(pl + 32 * 64) : l2;
            *reinterpret_cast<uint4*>(smem + KTILE_BYTES + c.sk0) = l0;
            if (SP == 2) *reinterpret_cast<uint4*>(smem + KTILE_BYTES + c.sk1) = l1;
            *reinterpret_cast<uint4*>(smem + KS + KTILE_BYTES + c.sk0) = l2;
            if (SP == 2) *reinterpret_cast<uint4*>(smem + KS + KTILE_BYTES + c.sk1) = l3;
            char* vl = vw + VLO;
            *reinterpret_cast<uint2*>(vl + c.sv0a) = make_uint2(w0.x, w0.y);
            *reinterpret_cast<uint2*>(vl + c.sv0b) = make_uint2(w0.z, w0.w);
            if (SP == 2) {
                *reinterpret_cast<uint2*>(vl + c.sv1a) = make_uint2(w1.x, w1.y);
                *reinterpret_cast<uint2*>(vl + c.sv1b) = make_uint2(w1.z, w1.w);
            }
        }
    }
    __syncthreads();
    ATT_T(1);
    const bool busy = qbase < nq;  // wave-uniform: some of its 32 queries are live
    f32x16 sA[QT], sB[QT];
    if (!(SPLIT && QT == 1) || busy) qk_half<SPLIT, QT>(smem, c, qf, qfl, 0, sA);
    f32x16 o[QT][2];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) { o[qt][0][i] = 0.f; o[qt][1][i] = 0.f; }
    float mrun[QT], lsum[QT][2];  // per lane half, two partial sums each
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) mrun[qt] = -INFINITY;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) { lsum[qt][0] = 0.f; lsum[qt][1] = 0.f; }
    uint4 stage[4 * QT];
    // stages unrolled by 3 (K and V ring slot of stage j = j % 3, compile-time)
#define PIPE_STAGE(J, R, LAST)                                                                 \
    {                                                                                          \
        pipe_half<0, LAST, R, SPLIT, QT>(J, sA, sB, c, qf, qfl, o, mrun, lsum, stage, (J) % 3, busy); \
        pipe_half<1, LAST, R, SPLIT, QT>(J, sB, sA, c, qf, qfl, o, mrun, lsum, stage, (J) % 3, busy); \
    }
    const int last = c.nkb - 1;
    int j = 0;
    for (; j + 3 <= last; j += 3) {
        PIPE_STAGE(j, 0, false)
        PIPE_STAGE(j + 1, 1, false)
        PIPE_STAGE(j + 2, 2, false)
    }
    if (j < last) {  // j % 3 == 0 here
        PIPE_STAGE(j, 0, false)
        ++j;
        if (j < last) {
            PIPE_STAGE(j, 1, false)
            ++j;
        }
    }
    PIPE_STAGE(last, -1, true)  // slot last % 3 at run time
#undef PIPE_STAGE
    ATT_T(2);

    // O staged through LDS (the K / V rings are dead once every wave is past its last
    // stage) as this wave's [32 QT queries][64 d] bf16, 16-B chunk c of row r at c ^ (r & 7),
    // then written as whole 128-B row pieces: 8 rows per wave-instruction instead of 32
    // rows x 16 B (the store tail of a row-per-lane epilogue is issue-bound)
    __syncthreads();
    char* st = smem + wave * (32 * QT * 128);
    if constexpr (!SPLIT) {
        if (MLG_ATT_STAGE_W && QT == 2) {
            // lanes l / l + 32 hold the two 8-B halves of chunk (dt, g) of rows col (tile 0) and
            // 32 + col (tile 1): after the swap lane l < 32 holds row col's whole chunk, lane
            // l + 32 row 32 + col's -- one b128 write each, 8 consecutive rows per write group
            const float inv0 = 1.0f / swap_sum(lsum[0][0] + lsum[0][1]);
            const float inv1 = 1.0f / swap_sum(lsum[QT - 1][0] + lsum[QT - 1][1]);
            const int r = 32 * hh + col;
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x16& a0 = o[0][dt];
                    const f32x16& a1 = o[QT - 1][dt];
                    const auto s0 = __builtin_amdgcn_permlane32_swap(
                        pack_bf16x2(a0[4 * g] * inv0, a0[4 * g + 1] * inv0),
                        pack_bf16x2(a1[4 * g] * inv1, a1[4 * g + 1] * inv1), false, false);
                    const auto s1 = __builtin_amdgcn_permlane32_swap(
                        pack_bf16x2(a0[4 * g + 2] * inv0, a0[4 * g + 3] * inv0),
                        pack_bf16x2(a1[4 * g + 2] * inv1, a1[4 * g + 3] * inv1), false, false);
                    *reinterpret_cast<uint4*>(st + r * 128 + (((dt * 4 + g) ^ (r & 7)) << 4)) =
                        make_uint4(s0[0], s1[0], s0[1], s1[1]);
                }
        } else {
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const float inv = 1.0f / swap_sum(lsum[qt][0] + lsum[qt][1]);
                const int r = qt * 32 + col;
#pragma unroll
                for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        uint2 w;
                        w.x = pack_bf16x2(o[qt][dt][4 * g] * inv, o[qt][dt][4 * g + 1] * inv);
                        w.y = pack_bf16x2(o[qt][dt][4 * g + 2] * inv, o[qt][dt][4 * g + 3] * inv);
                        *reinterpret_cast<uint2*>(st + r * 128 + (((dt * 4 + g) ^ (r & 7)) << 4) + 8 * hh) = w;
                    }
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes landed
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int p = 0; p < 4 * QT; ++p) {
            const int r = p * 8 + (lane >> 3), c = lane & 7, qrow = qbase + r;
            if (qrow < nq)
                *reinterpret_cast<uint4*>(orow + (size_t)qrow * ldo + c * 8) =
                    *reinterpret_cast<const uint4*>(st + r * 128 + ((c ^ (r & 7)) << 4));
        }
    } else {  // two passes through the staging image: hi rows, then lo rows at column lo_col
        float inv[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) inv[qt] = 1.0f / swap_sum(lsum[qt][0] + lsum[qt][1]);
#pragma unroll
        for (int part = 0; part < 2; ++part) {
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const int r = qt * 32 + col;
#pragma unroll
                for (int dt = 0; dt < 2; ++dt) {
                    if (MLG_ATT_STAGE_W) {
                        // lanes l / l + 32 hold the two 8-B halves of chunks (dt, g) and (dt, g + 1)
                        // of row r: after the swap lane l < 32 holds chunk g whole, lane l + 32
                        // chunk g + 1 -- one conflict-free b128 write each (8 rows per write
                        // group) instead of two b64 writes whose rows r and r + 8 shared banks
#pragma unroll
                        for (int g = 0; g < 4; g += 2) {
                            uint2 w0, wl0, w1, wl1;
                            split_bf16x4(o[qt][dt][4 * g] * inv[qt], o[qt][dt][4 * g + 1] * inv[qt],
                                         o[qt][dt][4 * g + 2] * inv[qt], o[qt][dt][4 * g + 3] * inv[qt], w0, wl0);
                            split_bf16x4(o[qt][dt][4 * g + 4] * inv[qt], o[qt][dt][4 * g + 5] * inv[qt],
                                         o[qt][dt][4 * g + 6] * inv[qt], o[qt][dt][4 * g + 7] * inv[qt], w1, wl1);
                            const uint2 a = part ? wl0 : w0, b = part ? wl1 : w1;
                            const auto s0 = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
                            const auto s1 = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
                            const int gg = g + hh;
                            *reinterpret_cast<uint4*>(st + r * 128 + (((dt * 4 + gg) ^ (r & 7)) << 4)) =
                                make_uint4(s0[0], s1[0], s0[1], s1[1]);
                        }
                    } else {
#pragma unroll
                        for (int g = 0; g < 4; ++g) {
                            uint2 w, wl;
                            split_bf16x4(o[qt][dt][4 * g] * inv[qt], o[qt][dt][4 * g + 1] * inv[qt],
                                         o[qt][dt][4 * g + 2] * inv[qt], o[qt][dt][4 * g + 3] * inv[qt], w, wl);
                            *reinterpret_cast<uint2*>(st + r * 128 + (((dt * 4 + g) ^ (r & 7)) << 4) + 8 * hh) =
                                part ? wl : w;
                        }
                    }
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes landed
            __builtin_amdgcn_wave_barrier();
            bf16_t* dst = orow + (part ? lo_col : 0);
            // a vector type, not uint4: copies of the HIP struct are memcpys, which kept this
            // array out of registers (hipcc then placed it in LDS: 32 KiB per workgroup)
            u32x4 rows[4 * QT];
#pragma unroll
            for (int p = 0; p < 4 * QT; ++p) {
                const int r = p * 8 + (lane >> 3), c = lane & 7;
                rows[p] = *reinterpret_cast<const u32x4*>(st + r * 128 + ((c ^ (r & 7)) << 4));
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // staging read before the next part overwrites it
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int p = 0; p < 4 * QT; ++p) {
                const int r = p * 8 + (lane >> 3), c = lane & 7, qrow = qbase + r;
                if (qrow < nq) *reinterpret_cast<u32x4*>(dst + (size_t)qrow * ldo + c * 8) = rows[p];
            }
        }
    }
}

// Ragged batch: task t attends query rows [q_off, q_off + q_len) to keys / values
// [kv_off, kv_off + kv_len) of a flat token layout (offsets multiples of 64, rows
// zero-padded to the next multiple of 64); Q, K: [heads][Npad][64]; V^T tiled per 64-key
// block, [heads][Npad / 64][64 d][64 keys] (a plain [64][Npad] V^T would put each d-row
// of a block in a different 2 MB page at large Npad); output rows out_off + r of
// O [Npad][ldo] at column h * 64.
// 1-D grid of qblocks x heads x tasks (rounded up to a multiple of 8), dealt so that the
// query blocks of one (task, head) -- which all stream the same K / V^T -- land on one
// XCD (hardware deals linear block b to XCD b % 8) and share its L2.
// VIT: the same tile under a second symbol, so rocprof's per-kernel rows (and their
// average durations) keep the ViT's ~70 us launches apart from LightGlue's
template <bool VIT, bool SPLIT = false, int NW = 4>
__global__ __launch_bounds__(64 * NW, 1) void k_attention_varlen(const bf16_t* __restrict__ Q,
                                                             const bf16_t* __restrict__ K,
                                                             const bf16_t* __restrict__ Vt, bf16_t* __restrict__ O,
                                                             int ldo, int Npad, const int4* __restrict__ tasks,
                                                             const int* __restrict__ out_off, int nqb, int heads,
                                                             int total, size_t lo_off, int lo_col) {
    __shared__ __attribute__((aligned(16))) char smem[3 * Slots<SPLIT>::K + 3 * Slots<SPLIT>::V];
    const int per_xcd = (int)gridDim.x >> 3;
    const int logical = ((int)blockIdx.x & 7) * per_xcd + ((int)blockIdx.x >> 3);
    if (logical >= total) return;
    const int qb = logical % nqb;
    const int h = (logical / nqb) % heads;
    const int t = logical / (nqb * heads);
    const int4 tk = tasks[t];  // q_off, q_len, kv_off, kv_len
    if (qb * 256 >= tk.y || tk.w <= 0) return;
    const int qpad = (tk.y + 63) & ~63;
    unsigned long long att_tt[4] = {};
    ATT_T(0);
    attention_tile_pipe<SPLIT, NW>(att_tt, smem, Q + ((size_t)h * Npad + tk.x) * 64, K + ((size_t)h * Npad + tk.z) * 64,
                               Vt + ((size_t)h * Npad + tk.z) * 64, tk.w, tk.y, qpad, qb,
                               O + (size_t)out_off[t] * ldo + h * 64, ldo, lo_off, lo_col);
#if MLG_ATT_TRACE
    if (!VIT && threadIdx.x == 0 && logical < ATT_TRACE_WGS) {
        ATT_T(3);
        unsigned long long* o = g_att_trace + (size_t)logical * 8;
        for (int i = 0; i < 4; ++i) o[i] = att_tt[i];
        o[4] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID
        o[5] = (unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
        o[6] = (unsigned long long)tk.y;
        o[7] = 1;
    }
#endif
    (void)att_tt;
}

// ViT tasks: image b attends its own segment [b * Tpad, b * Tpad + T) in every head;
// output rows b * T ..
__global__ void k_vit_tasks(int4* __restrict__ tasks, int* __restrict__ out_off, int B, int T, int Tpad) {
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
        tasks[b] = make_int4(b * Tpad, T, b * Tpad, T);
        out_off[b] = b * T;
    }
}

template <bool VIT, bool SPLIT = false, int NW = 4>
int varlen_launch(const bf16_t* Q, const bf16_t* K, const bf16_t* Vt, bf16_t* O, int ldo, int Npad, int heads,
                  const int4* tasks, const int* out_off, int ntasks, int max_q, hipStream_t s, size_t lo_off = 0,
                  int lo_col = 0) {
    if (ntasks <= 0) return MLG_OK;
    if (Npad % 64 || heads <= 0 || max_q <= 0) return MLG_EINVAL;
    const int nqb = (max_q + 255) / 256;
    const long total = (long)nqb * heads * ntasks;
    if (total > (1L << 30)) return MLG_EINVAL;
    const int grid = (int)((total + 7) & ~7L);
    hipLaunchKernelGGL((k_attention_varlen<VIT, SPLIT, NW>), dim3(grid), dim3(64 * NW), 0, s, Q, K, Vt, O, ldo, Npad, tasks,
                       out_off, nqb, heads, (int)total, lo_off, lo_col);
    MLG_LAUNCH_CHECK();
    return MLG_OK;
}

}  // namespace

// copies the phase trace of a MLG_ATT_TRACE build ([65536][8] u64, by logical workgroup:
// 4 stamps, HW_ID, XCC_ID, query count, written flag); -1 otherwise
extern "C" int mlg_dbg_att_trace(void* host, size_t bytes) {
#if MLG_ATT_TRACE
    const size_t n = bytes < sizeof(g_att_trace) ? bytes : sizeof(g_att_trace);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_att_trace), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : MLG_EHIP;
#else
    (void)host;
    (void)bytes;
    return MLG_EINVAL;
#endif
}

int mlg_attention(const bf16_t* Q, const bf16_t* K, const bf16_t* Vt, bf16_t* O, int B, int T, int Tpad,
                  int32_t* task_ws, hipStream_t s) {
    if (B <= 0 || T <= 0 || Tpad % 64 || Tpad < T || !task_ws || (long)B * Tpad * 64 >= (1L << 31)) return MLG_EINVAL;
    int4* tasks = reinterpret_cast<int4*>(task_ws);
    int* out_off = task_ws + 4 * B;
    hipLaunchKernelGGL(k_vit_tasks, dim3(1), dim3(256), 0, s, tasks, out_off, B, T, Tpad);
    MLG_LAUNCH_CHECK();
    return varlen_launch<true>(Q, K, Vt, O, 768, B * Tpad, 12, tasks, out_off, B, T, s);
}

// Split-bf16 ViT attention (MLG_VIT_SPLIT): Q, K, Vt hi planes with the lo planes
// lo_off elements further; O rows of 1536 = [hi | lo].  MLG_ATTN_SPLIT_WAVES: 4 (64 queries
// per wave, one wave per SIMD: 288 registers) or 8 (32 per wave, two per SIMD).
#ifndef MLG_ATTN_SPLIT_WAVES
#define MLG_ATTN_SPLIT_WAVES 8
#endif
int mlg_attention_split(const bf16_t* Q, const bf16_t* K, const bf16_t* Vt, bf16_t* O, int B, int T, int Tpad,
                        size_t lo_off, int32_t* task_ws, hipStream_t s) {
    if (B <= 0 || T <= 0 || Tpad % 64 || Tpad < T || !task_ws || (long)B * Tpad * 64 >= (1L << 31)) return MLG_EINVAL;
    int4* tasks = reinterpret_cast<int4*>(task_ws);
    int* out_off = task_ws + 4 * B;
    hipLaunchKernelGGL(k_vit_tasks, dim3(1), dim3(256), 0, s, tasks, out_off, B, T, Tpad);
    MLG_LAUNCH_CHECK();
    return varlen_launch<true, true, MLG_ATTN_SPLIT_WAVES>(Q, K, Vt, O, 1536, B * Tpad, 12, tasks, out_off, B, T, s,
                                                          lo_off, 768);
}

// LightGlue: MLG_ATTN_LG_WAVES = 4 (64 queries per wave; two workgroups per CU give two
// waves per SIMD) or 8 (build-time A/B arm)
#ifndef MLG_ATTN_LG_WAVES
#define MLG_ATTN_LG_WAVES 4
#endif
int mlg_attention_varlen(const bf16_t* Q, const bf16_t* K, const bf16_t* Vt, bf16_t* O, int ldo, int Npad, int heads,
                         const int4* tasks, const int* out_off, int ntasks, int max_q, hipStream_t s) {
    return varlen_launch<false, false, MLG_ATTN_LG_WAVES>(Q, K, Vt, O, ldo, Npad, heads, tasks, out_off, ntasks, max_q,
                                                          s);
}
