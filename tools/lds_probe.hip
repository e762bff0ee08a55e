// LDS bank-conflict calibration on gfx950 (GPU box tool; VERDICT r04 "next 4/5": find the
// conflicting LDS access of the projection / attention / FFN kernels).
//
// One kernel per access pattern, each the exact lane -> address map of one LDS stream of
// the product kernels (attention.hip, lg_proj.hip, lg_ffn.hip), plus calibration
// patterns with a known conflict degree.  Run under
//   rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -- ./lds_probe
// the counters per kernel give each stream's conflict cycles per instruction.
//   hipcc -O3 --offload-arch=gfx950 -o lds_probe tools/lds_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITERS = 4096;
constexpr int LDS_BYTES = 64 * 1024;

// access widths
enum { R16 = 0, R8 = 1, W16 = 2, W8 = 3, R4 = 4, R1 = 5 };

struct Lane {
    int tid, lane, wave, col, hh;
};

// ------------------------------------------------------------------ patterns
// each returns the byte offset of this lane's access at iteration `it`
__device__ __forceinline__ int p_contig16(const Lane& l, int) { return l.lane * 16; }
__device__ __forceinline__ int p_contig8(const Lane& l, int) { return l.lane * 8; }
__device__ __forceinline__ int p_stride256_16(const Lane& l, int) { return (l.lane * 256) & (LDS_BYTES - 1); }
__device__ __forceinline__ int p_stride128_8(const Lane& l, int) { return (l.lane * 128) & (LDS_BYTES - 1); }
__device__ __forceinline__ int p_2way8(const Lane& l, int) { return (l.lane & 31) * 8 + (l.lane >> 5) * 256; }

// attention.hip
__device__ __forceinline__ int k_off(int key, int chunk) { return key * 128 + ((chunk ^ ((key >> 1) & 7)) << 4); }
__device__ __forceinline__ int v_off(int d, int gran) { return d * 128 + ((gran ^ (((d >> 1) ^ (d >> 5)) & 15)) << 3); }
__device__ __forceinline__ int p_attn_k_read(const Lane& l, int it) {  // qk_half: ds_read_b128
    const int st = it & 3, kt = (it >> 2) & 1;
    return kt * 4096 + k_off(l.col, 2 * st + l.hh);
}
__device__ __forceinline__ int p_attn_v_read(const Lane& l, int it) {  // pipe_half: ds_read_b64
    const int dt = it & 1, st = (it >> 1) & 1, h = (it >> 2) & 1, hi = (it >> 3) & 1;
    return 8192 + v_off(dt * 32 + l.col, h * 8 + st * 4 + l.hh + 2 * hi);
}
__device__ __forceinline__ int p_attn_k_write(const Lane& l, int it) {  // stage -> K ring, b128
    const int srow = l.tid >> 3, sch = l.tid & 7;
    return k_off(srow + 32 * (it & 1), sch);
}
__device__ __forceinline__ int p_attn_v_write(const Lane& l, int it) {  // stage -> V ring, b64
    const int srow = l.tid >> 3, sch = l.tid & 7;
    return 8192 + v_off(srow + 32 * ((it >> 1) & 1), 2 * sch + (it & 1));
}
__device__ __forceinline__ int p_attn_o_write(const Lane& l, int it) {  // O staging, b64
    const int qt = it & 1, dt = (it >> 1) & 1, g = (it >> 2) & 3, r = qt * 32 + l.col;
    return l.wave * 8192 + r * 128 + (((dt * 4 + g) ^ (r & 7)) << 4) + 8 * l.hh;
}
// lg_proj.hip (pipelined resident form)
__device__ __forceinline__ int xoff(int row, int chunk) { return row * 512 + ((chunk ^ (row & 15)) << 4); }
__device__ __forceinline__ int stage_off(int h, int row, int e) {
    return (h * 64 + row) * 128 + ((((e >> 3) ^ (row & 7))) << 4) + (e & 7) * 2;
}
__device__ __forceinline__ int p_proj_x_read(const Lane& l, int it) {  // res/pipe GEMM, b128
    const int ks = it & 15, mt = (it >> 4) & 1;
    return xoff(l.col + 32 * mt, 2 * ks + l.hh);
}
__device__ __forceinline__ int p_proj_fac_read(const Lane& l, int it) {  // slice_qk cos / sin, b64
    const int g = it & 3, mt = (it >> 2) & 1;
    const int n = 32 * l.wave + 8 * g + 4 * l.hh, r = 32 * mt + l.col, j = (n & 63) / 2;
    const int eo = r * 32 + 4 * ((j >> 2) ^ ((r >> 1) & 7)) + (j & 3);
    return 32768 + eo * 4;
}
__device__ __forceinline__ int p_proj_stage_qk(const Lane& l, int it) {  // slice_qk staging write, b64
    const int g = it & 3, mt = (it >> 2) & 1;
    const int n = 32 * l.wave + 8 * g + 4 * l.hh, h = n >> 6, d = n & 63, r = 32 * mt + l.col;
    return stage_off(h, r, d);
}
__device__ __forceinline__ int p_proj_stage_v(const Lane& l, int it) {  // slice_v staging write, b64
    const int g = it & 3, mt = (it >> 2) & 1;
    const int n = 32 * l.wave + l.col, h = n >> 6, d = n & 63, r = 32 * mt + 8 * g + 4 * l.hh;
    return stage_off(h, d, r);
}
__device__ __forceinline__ int p_proj_copyout(const Lane& l, int it) {  // copy_out64 read, b128
    const int L = (it & 3) * 512 + l.tid, h = L / 512, row = (L >> 3) & 63, c = L & 7;
    return stage_off(h, row, 8 * c);
}
// lg_proj.hip paired staging (MLG_PROJ_SWAP, round 5): b128 writes of whole chunks, b128 copy-out
// (pattern 29-31: the (r >> 1) & 7 swizzle first tried, 2-way on the writes; 36-38: r & 7, the product)
__device__ __forceinline__ int pair_off(int h, int row, int c) { return (h * 64 + row) * 128 + ((c ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int pair_off7(int h, int row, int c) { return (h * 64 + row) * 128 + ((c ^ (row & 7)) << 4); }
__device__ __forceinline__ int p_pair7_qk_write(const Lane& l, int it) {
    const int n = 32 * l.wave + 8 * (it & 3);
    return pair_off7(n >> 6, 32 * l.hh + l.col, (n & 63) >> 3);
}
__device__ __forceinline__ int p_pair7_v_write(const Lane& l, int it) {
    const int n = 32 * l.wave + l.col;
    return pair_off7(n >> 6, n & 63, (it & 3) + 4 * l.hh);
}
__device__ __forceinline__ int p_pair7_copyout(const Lane& l, int it) {
    const int L = (it & 3) * 512 + l.tid, h = L / 512, row = (L >> 3) & 63, c = L & 7;
    return pair_off7(h, row, c);
}
__device__ __forceinline__ int p_pair_qk_write(const Lane& l, int it) {  // stage_pair_qk, b128
    const int n = 32 * l.wave + 8 * (it & 3);
    return pair_off(n >> 6, 32 * l.hh + l.col, (n & 63) >> 3);
}
__device__ __forceinline__ int p_pair_v_write(const Lane& l, int it) {  // stage_pair_v, b128
    const int n = 32 * l.wave + l.col;
    return pair_off(n >> 6, n & 63, (it & 3) + 4 * l.hh);
}
__device__ __forceinline__ int p_pair_copyout(const Lane& l, int it) {  // copy_out64 read, b128
    const int L = (it & 3) * 512 + l.tid, h = L / 512, row = (L >> 3) & 63, c = L & 7;
    return pair_off(h, row, c);
}
__device__ __forceinline__ int p_bias_bcast(const Lane& l, int it) {  // slice_qk bias float4 (2 addresses)
    return 32768 + (32 * l.wave + 8 * (it & 3) + 4 * l.hh) * 4;
}
__device__ __forceinline__ int p_live_u8(const Lane& l, int it) {  // slice_qk live byte
    return 40960 + 32 * ((it >> 2) & 1) + l.col;
}
__device__ __forceinline__ int p_live_u32(const Lane& l, int it) {  // slice_v live dword
    return 40960 + 32 * ((it >> 2) & 1) + 8 * (it & 3) + 4 * l.hh;
}
__device__ __forceinline__ int p_fac_tile(const Lane& l, int it) {  // slice_qk rotary float4 (lg_fac4 tile)
    const int g = it & 3, mt = (it >> 2) & 1;
    const int n = 32 * l.wave + 8 * g + 4 * l.hh, r = 32 * mt + l.col, p = (n & 63) >> 2;
    return 16384 + ((p * 64 + r) << 4);
}
// lg_ffn.hip
__device__ __forceinline__ int cat_off(int row, int chunk) { return row * 1024 + ((chunk ^ (row & 15)) << 4); }
__device__ __forceinline__ int p_ffn_cat_read(const Lane& l, int it) {  // gemm_phase, b128
    const int ks = it & 31, mt = (it >> 5) & 1;
    return cat_off(l.col + 32 * mt, 2 * ks + l.hh);
}
__device__ __forceinline__ int p_ffn_cat_write(const Lane& l, int it) {  // GELU / msg epilogue write, b64
    const int t = it & 3, g = (it >> 2) & 3, mt = (it >> 4) & 1;
    const int n = 128 * (l.wave & 3) + 32 * t + 8 * g + 4 * l.hh;
    return cat_off(32 * mt + l.col, n / 8) + 8 * l.hh;
}
__device__ __forceinline__ int p_ffn_y_write(const Lane& l, int it) {  // ffn2 f32 staging, b128
    const int t = it & 1, g = (it >> 1) & 3, mt = (it >> 3) & 1;
    const int n = 64 * (l.wave & 3) + 32 * t + 8 * g + 4 * l.hh, r = 32 * mt + l.col;
    return r * 1024 + (((n >> 2) ^ (r & 15)) << 4);
}
__device__ __forceinline__ int p_ffn_y_read(const Lane& l, int it) {  // residual row pass, b128
    const int r = (l.wave & 3) * 16 + (it & 15);
    return r * 1024 + ((l.lane ^ (r & 15)) << 4);
}

// write-rule calibration (b64): which lane groups share a cycle, what conflicts
__device__ __forceinline__ int p_w_swap8(const Lane& l, int) { return (l.lane * 8) ^ 8; }
__device__ __forceinline__ int p_w_stride16(const Lane& l, int) { return l.lane * 16; }
__device__ __forceinline__ int p_w_gap64(const Lane& l, int) { return l.lane * 8 + (l.lane >> 3) * 64; }
__device__ __forceinline__ int p_w_swap16(const Lane& l, int) { return (l.lane * 8) ^ (((l.lane >> 3) & 1) * 16); }
__device__ __forceinline__ int p_w_it(const Lane& l, int it) { return l.lane * 8 + (it & 1) * 512; }
__device__ __forceinline__ int p_w_rev(const Lane& l, int) { return (63 - l.lane) * 8; }
__device__ __forceinline__ int p_w_half(const Lane& l, int) { return (l.lane & 31) * 8 + (l.lane >> 5) * 4096; }
__device__ __forceinline__ int p_w_rows(const Lane& l, int) {  // 8 lanes per 128-B row, rows 128 B apart, in order
    return (l.lane >> 3) * 128 + (l.lane & 7) * 16;
}
__device__ __forceinline__ int p_w_rows8(const Lane& l, int) {  // 16 lanes per 128-B row (contiguous)
    return (l.lane >> 4) * 128 + (l.lane & 15) * 8;
}
__device__ __forceinline__ int p_w_xor(const Lane& l, int) {  // contiguous 8-B granules, XOR-permuted per 128 B
    const int row = l.lane >> 4, g = l.lane & 15;
    return row * 128 + ((g ^ (row & 15)) << 3);
}

template <int PAT>
__device__ __forceinline__ int addr_of(const Lane& l, int it) {
    switch (PAT) {
        case 0: return p_contig16(l, it);
        case 1: return p_contig8(l, it);
        case 2: return p_stride256_16(l, it);
        case 3: return p_stride128_8(l, it);
        case 4: return p_2way8(l, it);
        case 5: return p_attn_k_read(l, it);
        case 6: return p_attn_v_read(l, it);
        case 7: return p_attn_k_write(l, it);
        case 8: return p_attn_v_write(l, it);
        case 9: return p_attn_o_write(l, it);
        case 10: return p_proj_x_read(l, it);
        case 11: return p_proj_fac_read(l, it);
        case 12: return p_proj_stage_qk(l, it);
        case 13: return p_proj_stage_v(l, it);
        case 14: return p_proj_copyout(l, it);
        case 15: return p_ffn_cat_read(l, it);
        case 16: return p_ffn_cat_write(l, it);
        case 17: return p_ffn_y_write(l, it);
        case 18: return p_ffn_y_read(l, it);
        case 19: return p_w_swap8(l, it);
        case 20: return p_w_stride16(l, it);
        case 21: return p_w_gap64(l, it);
        case 22: return p_w_swap16(l, it);
        case 23: return p_w_it(l, it);
        case 24: return p_w_rev(l, it);
        case 25: return p_w_half(l, it);
        case 26: return p_w_rows(l, it);
        case 27: return p_w_rows8(l, it);
        case 28: return p_w_xor(l, it);
        case 29: return p_pair_qk_write(l, it);
        case 30: return p_pair_v_write(l, it);
        case 31: return p_pair_copyout(l, it);
        case 32: return p_bias_bcast(l, it);
        case 33: return p_live_u8(l, it);
        case 34: return p_live_u32(l, it);
        case 35: return p_fac_tile(l, it);
        case 36: return p_pair7_qk_write(l, it);
        case 37: return p_pair7_v_write(l, it);
        case 38: return p_pair7_copyout(l, it);
    }
    return 0;
}

// one LDS access per iteration; the address depends on `it` through a runtime value so
// the compiler cannot merge two accesses into a ds_read2 / ds_write2
template <int PAT, int MODE>
__global__ __launch_bounds__(256) void k_probe(uint32_t* __restrict__ sink, int salt) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    Lane l;
    l.tid = threadIdx.x;
    l.lane = threadIdx.x & 63;
    l.wave = threadIdx.x >> 6;
    l.col = l.lane & 31;
    l.hh = l.lane >> 5;
    for (int i = threadIdx.x; i < LDS_BYTES / 4; i += 256) reinterpret_cast<uint32_t*>(lds)[i] = i ^ salt;
    __syncthreads();
    uint32_t acc = 0;
    uint4 v4 = make_uint4(salt, salt + 1, salt + 2, salt + 3);
#pragma unroll 8
    for (int it = 0; it < ITERS; ++it) {
        constexpr int W = (MODE == R16 || MODE == W16) ? 16 : (MODE == R4 ? 4 : (MODE == R1 ? 1 : 8));
        const int a = addr_of<PAT>(l, it ^ (salt & 0x10000)) & (LDS_BYTES - W);
        if (MODE == R16) {
            const uint4 v = *reinterpret_cast<const uint4*>(lds + a);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else if (MODE == R8) {
            const uint2 v = *reinterpret_cast<const uint2*>(lds + a);
            acc += v.x ^ v.y;
        } else if (MODE == W16) {
            v4.x += it;
            *reinterpret_cast<uint4*>(lds + a) = v4;
        } else if (MODE == W8) {
            v4.x += it;
            *reinterpret_cast<uint2*>(lds + a) = make_uint2(v4.x, v4.y);
        } else if (MODE == R1) {
            acc += (uint32_t)(uint8_t)lds[a];
        } else {
            acc += *reinterpret_cast<const uint32_t*>(lds + a);
        }
        asm volatile("" ::: "memory");  // no merging of consecutive accesses into ds_*2 forms
    }
    __syncthreads();
    if (MODE == W16 || MODE == W8) acc = reinterpret_cast<const uint32_t*>(lds)[threadIdx.x];
    if (acc == 0x9e3779b9u) sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int PAT, int MODE>
void run(const char* name, uint32_t* sink) {
    hipLaunchKernelGGL((k_probe<PAT, MODE>), dim3(1024), dim3(256), 0, 0, sink, 7);
    hipError_t e = hipDeviceSynchronize();
    printf("%-24s pattern %2d mode %d: %s\n", name, PAT, MODE, e == hipSuccess ? "ok" : hipGetErrorString(e));
}

int main() {
    uint32_t* sink = nullptr;
    if (hipMalloc(&sink, 1024 * 256 * 4) != hipSuccess) return 1;
    run<0, R16>("contig_b128", sink);
    run<1, R8>("contig_b64", sink);
    run<2, R16>("stride256_b128(16way)", sink);
    run<3, R8>("stride128_b64", sink);
    run<4, R8>("two_way_b64", sink);
    run<5, R16>("attn_k_read", sink);
    run<6, R8>("attn_v_read", sink);
    run<7, W16>("attn_k_write", sink);
    run<8, W8>("attn_v_write", sink);
    run<9, W8>("attn_o_write", sink);
    run<10, R16>("proj_x_read", sink);
    run<11, R8>("proj_fac_read", sink);
    run<12, W8>("proj_stage_qk_write", sink);
    run<13, W8>("proj_stage_v_write", sink);
    run<14, R16>("proj_copyout_read", sink);
    run<15, R16>("ffn_cat_read", sink);
    run<16, W8>("ffn_cat_write", sink);
    run<17, W16>("ffn_y_write", sink);
    run<18, R16>("ffn_y_read", sink);
    run<0, W16>("contig_w128", sink);
    run<1, W8>("contig_w64", sink);
    run<19, W8>("w_swap8", sink);
    run<20, W8>("w_stride16", sink);
    run<21, W8>("w_gap64", sink);
    run<22, W8>("w_swap16", sink);
    run<23, W8>("w_it", sink);
    run<24, W8>("w_rev", sink);
    run<25, W8>("w_half", sink);
    run<26, W8>("w_rows(8/row,16B)", sink);
    run<27, W8>("w_rows8", sink);
    run<28, W8>("w_xor", sink);
    run<8, R8>("attn_v_write_as_read", sink);
    run<12, R8>("proj_stage_qk_as_read", sink);
    run<20, R8>("r_stride16", sink);
    run<1, W16>("contig8_as_w128", sink);
    run<29, W16>("pair_qk_write", sink);
    run<30, W16>("pair_v_write", sink);
    run<31, R16>("pair_copyout_read", sink);
    run<32, R16>("bias_bcast_read", sink);
    run<33, R1>("live_u8_read", sink);
    run<34, R4>("live_u32_read", sink);
    run<35, R16>("fac_tile_read", sink);
    run<36, W16>("pair7_qk_write", sink);
    run<37, W16>("pair7_v_write", sink);
    run<38, R16>("pair7_copyout_read", sink);
    (void)hipFree(sink);
    return 0;
}
