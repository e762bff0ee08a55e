// Internal (C++ linkage) launchers of the mlgate HIP kernels.  The public C ABI is
// include/mlgate.h; these are the building blocks behind it.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <algorithm>

typedef uint16_t bf16_t;

// The head every struct argument of the C ABI begins with (include/mlgate.h
// MLG_STRUCT_INIT): true iff it names this struct's size and the library's ABI version.
template <class T>
inline bool mlg_head_ok(const T* p, uint32_t abi_version) {
    return p && p->struct_size == (uint32_t)sizeof(T) && p->abi_version == abi_version;
}

// HIP-event profiling scope (abi.cpp): records the launches between construction and
// destruction on stream s into `slot` with `work` algorithmic FLOPs (or bytes).
// Slots: 0 fc1, 1 fc2, 2 qkv, 3 proj, 4 ViT attention, 5 LightGlue attention,
// 6 LightGlue q/k/v projections, 7 SuperPoint 3x3 convs, 8 LightGlue fused block tail
// (lg_ffn.hip; its `work` is algorithmic HBM bytes, the others' FLOPs).
#define MLG_PROF_SLOTS 9
struct MlgProfScope {
    int slot;
    hipStream_t s;
    double work;
    hipEvent_t a = nullptr, b = nullptr;
    MlgProfScope(int slot, hipStream_t s, double work);
    ~MlgProfScope();
};

// gemm_bf16.hip -- C = epi(A[M,K] . W[N,K]^T), N % 128 == 0, K % 64 == 0
int mlg_gemm_f32out(const bf16_t* A, const bf16_t* W, float* C, int M, int N, int K, hipStream_t s);
int mlg_gemm_f32out_variant(int variant, const bf16_t* A, const bf16_t* W, float* C, int M, int N, int K,
                            hipStream_t s);
int mlg_gemm_set_variant(int variant);
// leading-dimension variants (A row stride lda, output row stride ldc / ldx)
int mlg_gemm_bias_f32_ld(const bf16_t* A, int lda, const bf16_t* W, const float* bias, float* C, int ldc, int M,
                         int N, int K, hipStream_t s);
// C = A . W^T + bias split into bf16 hi / lo halves (C = hi + lo to 2^-17 relative),
// stored k-step-major [N / 16][M][16] (LightGlue assignment operands)
int mlg_gemm_bias_split_bf16(const bf16_t* A, int lda, const bf16_t* W, const float* bias, bf16_t* H, bf16_t* L,
                             int M, int N, int K, hipStream_t s);
int mlg_gemm_bias_relu_bf16(const bf16_t* A, int lda, const bf16_t* W, const float* bias, bf16_t* C, int ldc,
                            int nvalid, int M, int N, int K_, hipStream_t s);
int mlg_gemm_bias_add_relu(const bf16_t* A, int lda, const bf16_t* W, const float* bias, const float* R, float* X,
                           int ldx, bf16_t* C, int M, int N, int K_, hipStream_t s);
// y = A . W^T (+ bias) (+ R) -> act (1 relu, 2 leaky 0.01, 3 elu + 1 on cols < act_cols)
// (vdiv != 0: cols >= act_cols / vdiv) -> f32 X and / or bf16 C (LoFTR convs on im2col rows
// and its transformer linears)
int mlg_gemm_conv(const bf16_t* A, int lda, const bf16_t* W, const float* bias, const float* R, int ldr, float* X,
                  int ldx, bf16_t* C, int ldc, int act, int act_cols, int M, int N, int K_, hipStream_t s,
                  float vdiv = 0.f);
// LoFTR's FPN merge fused into the lateral 1x1 conv: C = bf16((A W^T + bias) + up(src)),
// src the coarser NHWC f32 map [B, h, w, N], M = B (2h) (2w) output pixels (k_lf_up_add's
// arithmetic in the epilogue)
int mlg_gemm_conv_upadd(const bf16_t* A, int lda, const bf16_t* W, const float* bias, const float* src, int h, int w,
                        bf16_t* C, int M, int N, int K_, hipStream_t s);
// implicit-GEMM k x k (k = 1 or 3, pad k / 2) stride-s convolution over NHWC bf16 [B, H, W, C]
// (C % 64 == 0), weights [N][tap * C + c], EpiConv epilogue; `zero` = 16 zero bytes
int mlg_conv_implicit(const bf16_t* in, const bf16_t* zero, int B, int H, int W, int C, int k, int s,
                      const bf16_t* Wt, const float* bias, const float* R, int ldr, float* X, int ldx, bf16_t* Cout,
                      int ldc, int act, int act_cols, int N, hipStream_t st);
int mlg_attention_varlen(const bf16_t* Q, const bf16_t* K, const bf16_t* Vt, bf16_t* O, int ldo, int Npad, int heads,
                         const int4* tasks, const int* out_off, int ntasks, int max_q, hipStream_t s);
int mlg_gemm_bias_bf16(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* C, int M, int N, int K,
                       hipStream_t s);
int mlg_gemm_bias_gelu_bf16(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* C, int M, int N, int K,
                            hipStream_t s);
int mlg_gemm_residual(const bf16_t* A, const bf16_t* W, const float* bias, const float* gamma, float* X, int M,
                      int N, int K, hipStream_t s);
int mlg_gemm_qkv(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* Q, bf16_t* K, bf16_t* Vt, int M,
                 int T, int Tpad, hipStream_t s);
int mlg_gemm_patch(const bf16_t* A, const bf16_t* W, const float* bias, const float* pos, float* X, int M, int P,
                   int Kpad, hipStream_t s);

// attention.hip
// ViT self-attention through k_attention_varlen (Q, K [12][B * Tpad][64], V^T tiled
// [12][B * Tpad / 64][64][64], O [B * T][768]); task_ws: 5 * B int32 of device memory
int mlg_attention(const bf16_t* Q, const bf16_t* K, const bf16_t* Vt, bf16_t* O, int B, int T, int Tpad,
                  int32_t* task_ws, hipStream_t s);

// vit_ops.hip
int mlg_preprocess_patches(const uint8_t* img, int B, int H, int W, int C, long img_stride, int S, int Kpad,
                           int swap_rb, bf16_t* out, hipStream_t s, int split = 0);
int mlg_cls_rows(float* X, const float* cls, const float* pos, int B, int T, hipStream_t s);
int mlg_layernorm_bf16(const float* X, const float* g, const float* b, bf16_t* Y, int M, hipStream_t s);
// split-bf16 forward (MLG_VIT_SPLIT): [hi | lo] operand rows, weights [W_hi | W_lo] (2x the reduction dim)
int mlg_layernorm_split(const float* X, const float* g, const float* b, bf16_t* Y, int M, hipStream_t s);
int mlg_gemm_qkv_split(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* Q, bf16_t* K, bf16_t* Vt, int M,
                       int T, int Tpad, size_t lo_off, hipStream_t s);
int mlg_gemm_residual_split(const bf16_t* A, const bf16_t* W, const float* bias, const float* gamma, float* X, int M,
                            int N, int K0, hipStream_t s);
int mlg_gemm_bias_gelu_split(const bf16_t* A, const bf16_t* W, const float* bias, bf16_t* C, int M, int N, int K0,
                             hipStream_t s);
int mlg_gemm_patch_split(const bf16_t* A, const bf16_t* W, const float* bias, const float* pos, float* X, int M, int P,
                         int Kpad, hipStream_t s);
int mlg_attention_split(const bf16_t* Q, const bf16_t* K, const bf16_t* Vt, bf16_t* O, int B, int T, int Tpad,
                        size_t lo_off, int32_t* task_ws, hipStream_t s);
int mlg_final_norm_gem(const float* X, const float* g, const float* b, float* local, float* partial, float* desc,
                       int B, int T, int mean_pool, hipStream_t s);
size_t mlg_gem_partial_bytes(int B);

// salad.hip -- SALAD head per frame (token MLP, Sinkhorn, aggregation, normalisation)
int mlg_salad_head(const bf16_t* xn, const float* Y, int B, int T, const float* wt1, const float* bt1,
                   const float* wt2, const float* bt2, float dust, float* desc, hipStream_t s);

// knn.hip
int mlg_row_normalize(const float* X, float* Xn, int N, int D, float* norms, hipStream_t s);
int mlg_similarity_f32(const float* A, int Q, const float* B, int N, int D, float* S, int lds, hipStream_t s);
// the same product stored as LoFTR's coarse similarity (S / 256) / 0.1
int mlg_similarity_f32_loftr(const float* A, int Q, const float* B, int N, int D, float* S, int lds, hipStream_t s);
// the same similarity from split-bf16 operands (A / B rows [hi | lo], K0 = 256 each; B
// readable up to Npad = ncols rounded up to 256 rows): 3 bf16 MFMA products per product.
// nb > 1: nb pairs in one launch, pair z's operands at A / B + z pstride elements and its
// similarity at S + z M lds (one persistent tile queue for the whole pair group)
int mlg_gemm_sim_split_loftr(const bf16_t* A, const bf16_t* B, int M, int Npad, int K0, float* S, int lds, int ncols,
                             hipStream_t s, int nb = 1, long pstride = 0);
int mlg_similarity_f32_t(const float* A, int Q, const float* B, int N, int D, float* S, int lds, float* St, int ldt,
                         hipStream_t s);
int mlg_topk_gate(const float* S, int lds, int N, int Q, const double* tq, const double* tdb, const int64_t* fq,
                  const uint8_t* hfq, const int64_t* fdb, const uint8_t* hfdb, double min_gap, float thr, int k,
                  int gating, int32_t* idx, float* sim, uint8_t* valid, int32_t* count, unsigned long long* totals,
                  hipStream_t s);
int mlg_xcorr_reduce(const float* C, int n1, int n2, float* out, hipStream_t s);
size_t mlg_xcorr_batch_ws_bytes(int F, int L, int D, int P);
int mlg_xcorr_batch_run(const float* feats, int F, int L, int D, const int32_t* qa, const int32_t* qb, int P,
                        void* ws, size_t ws_bytes, float* score, hipStream_t s);
// fused kNN (k <= 32): no [Q, N] matrix; workspace mlg_knn_fused_ws_bytes(Q, N, k)
int mlg_row_normalize_wave(const float* X, float* Xn, int N, int D, float* norms, hipStream_t s);
int mlg_knn_fused_splits(int Q, int N);
size_t mlg_knn_fused_ws_bytes(int Q, int N, int k);
int mlg_knn_fused(const float* Xq, int Q, const float* Xd, int N, int D, const double* tq, const double* tdb,
                  const int64_t* fq, const uint8_t* hfq, const int64_t* fdb, const uint8_t* hfdb, double min_gap,
                  float thr, int k, int gating, void* ws, int32_t* idx, float* sim, uint8_t* valid, int32_t* count,
                  unsigned long long* totals, hipStream_t s);

// proximity.hip -- trajectory-proximity candidates + floor gate
bool mlg_proximity_shape_ok(int N, int row0, int nrows);
size_t mlg_proximity_ws_bytes(int N, int nrows);
int mlg_proximity_count_run(const double* pos, const int64_t* floor, int N, int row0, int nrows, double radius,
                            int min_gap, int strict, void* ws, size_t ws_bytes, long long* totals, hipStream_t s);
int mlg_proximity_emit_run(const double* pos, const int64_t* floor, int N, int row0, int nrows, double radius,
                           int min_gap, int strict, const void* ws, size_t ws_bytes, int32_t* pairs, double* dist,
                           uint8_t* valid, hipStream_t s);

// ransac.hip -- batched epipolar RANSAC + recoverPose
size_t mlg_ransac_ws_bytes(int P, long S_total, int H);
int mlg_ransac_run(const float* kp1, const float* kp2, const int32_t* offs, int P, long S_total, const double* K,
                   int k_stride, double thr, int H, uint64_t seed, void* ws, size_t ws_bytes, double* model_out,
                   uint8_t* mask, int32_t* inliers, double* pose, int32_t* status, hipStream_t s);
int mlg_recover_pose_run(const float* kp1, const float* kp2, const int32_t* offs, int P, const double* K,
                         int k_stride, const double* E, const uint8_t* mask, double* pose, hipStream_t s);

// superpoint.hip -- SuperPoint detector / descriptor
struct mlg_sp_weights_i {
    const float* conv1a_w;  // f32 [64][9]
    const float* conv1a_b;  // f32 [64]
    const bf16_t* w[11];    // conv1b conv2a conv2b conv3a conv3b conv4a conv4b convPa convPb convDa convDb
    const float* b[11];
};
size_t mlg_superpoint_ws_bytes(int B, int H, int W);
int mlg_superpoint_run(const mlg_sp_weights_i& w, const uint8_t* frames, int B, int H, int W, int C, long frame_stride,
                       float det_thr, int max_kp, int nms_radius, int border, void* ws, size_t ws_bytes, float* kpts,
                       float* kscores, float* desc, uint16_t* desc_bf16, int32_t* count, hipStream_t s);

// lightglue.hip -- LightGlue matcher over a ragged batch of pairs
struct mlg_lg_block_i {
    const bf16_t* Wqkv; const float* bqkv;  // self: [768][256]; cross: [to_qk; to_v] [512][256] (k-step-major)
    const bf16_t* Wout; const float* bout;  // [256][256]   } packed k-step-major,
    const bf16_t* Wf1;  const float* bf1;   // [512][512]   } [K/16][N][16] (lg_ffn.hip)
    const float* ln_g;  const float* ln_b;  // [512]
    const bf16_t* Wf2;  const float* bf2;   // [256][512]   }
};
struct mlg_lg_weights_i {
    const float* Wr;  // [32][2]
    mlg_lg_block_i self[9], cross[9];
    const bf16_t* Wfinal[9]; const float* bfinal[9];  // [256][256], [256]
    const float* wmatch[9];  const float* bmatch[9];  // [256], [1]
    const float* wconf[8];   const float* bconf[8];   // [256], [1]
    const float* ones;                                 // [256] of 1.0f
};
// lg_ffn.hip -- fused out_proj + FFN (Linear, LayerNorm, GELU, Linear) + residual of one
// LightGlue block over M token rows: X f32 [M][256] updated in place, its bf16 copy
// xcopy [M][ldc] (cols 0..255; read as the GEMM operand, then rewritten); ctx bf16
// [M][256] is the attention output.
// Optional heads fused into the block tail's final row pass (lightglue.hip k_lg_conf
// semantics): z = x . wm + bm -> lz = logsigmoid(z); with wc: conf = sigmoid(x . wc + bc),
// flags = (conf < thr) | (sigmoid(z) > 1 - width || conf <= thr) << 1; dead rows
// (rowseg < 0) get flags 0 and no lz.  wm == nullptr: off.
struct mlg_lg_conf_i {
    const int* rowseg;
    const float* wc; const float* bc;
    const float* wm; const float* bm;
    float thr, width;
    float* lz; uint8_t* flags;
};
// relu == 1: ReLU without LayerNorm (SuperGlue's MLP with BatchNorm folded into Wf1);
// relu == 2: a LoFTREncoderLayer tail (no biases; Wout = merge, then norm1; ReLU MLP; norm2
// before the residual; ln_g / ln_b = [norm1 | norm2], 256 each)
int mlg_lg_ffn(const bf16_t* ctx, float* X, bf16_t* xcopy, int ldc, int M, const mlg_lg_block_i& w, hipStream_t s,
               const mlg_lg_conf_i* conf = nullptr, int relu = 0);
// lg_proj.hip -- LightGlue q/k/v projections (+ rotary for the self block) straight into
// the attention operands; W packed k-step-major [16][768 | 512][16]; Npad % 64 == 0.
// efac: the rotary factors in the lg_fac4 layout (common.h), self block only
int mlg_lg_proj(bool self_block, const bf16_t* xcopy, int ldx, const bf16_t* W, const float* bias, const float* efac,
                const uint8_t* live, bf16_t* Q, bf16_t* K, bf16_t* Vt, int Npad, hipStream_t s);
// superglue.hip -- SuperGlue GNN + log-space optimal transport over a ragged batch of pairs
struct mlg_sg_weights_i {
    const float* kenc_w[3]; const float* kenc_b[3];
    const bf16_t* kenc_w4; const float* kenc_b4;
    const bf16_t* kenc_w5; const float* kenc_b5;
    mlg_lg_block_i layer[18];
    const bf16_t* Wfinal; const float* bfinal;
    float bin_score;
};
size_t mlg_superglue_ws_bytes(int P, int kmax);
int mlg_superglue_run(const mlg_sg_weights_i& w, const float* kpts, const float* kscores, const float* desc,
                      const int32_t* counts, int kmax, int W, int H, const int32_t* pa, const int32_t* pb, int P,
                      int iters, float thr, void* ws, size_t ws_bytes, int32_t* matches, float* mscores,
                      int32_t* nmatch, hipStream_t s);
size_t mlg_lightglue_ws_bytes(int P, int kmax);
int mlg_lightglue_run(const mlg_lg_weights_i& w, const float* kpts, const float* desc, const int32_t* counts, int kmax,
                      const int32_t* pa, const int32_t* pb, int P, float depth_conf, float width_conf,
                      float filter_thr, int pruning_min, void* ws, size_t ws_bytes, int32_t* matches, float* mscores,
                      int32_t* nmatch, int32_t* stop_layer, hipStream_t s);

// resnet.hip -- ResNet-50 GAP descriptor (MixVPR / SALAD fallback)
struct mlg_rn_block_i {
    const bf16_t* w1; const float* b1;  // conv1 1x1 [max(width,128)][Cin] (BN folded; pad rows zero)
    const bf16_t* w2; const float* b2;  // conv2 3x3 [max(width,128)][9 * width] (k = tap * width + c)
    const bf16_t* w3; const float* b3;  // conv3 1x1 [4 width][width]
    const bf16_t* wd; const float* bd;  // downsample 1x1 [4 width][Cin] or NULL
};
struct mlg_rn_weights_i {
    const float* stem_w;  // f32 [64][7][7][3] (BN folded)
    const float* stem_b;  // f32 [64]
    mlg_rn_block_i blocks[16];
};
size_t mlg_resnet50_ws_bytes(int B, int H, int W);
// resized_u8 != NULL: only the Pillow resize runs, into [B, 224, 224, 3] (parity entry)
int mlg_resnet50_run(const mlg_rn_weights_i& w, const uint8_t* frames, int B, int H, int W, int C, long frame_stride,
                     int D, void* ws, size_t ws_bytes, float* desc, uint8_t* resized_u8, hipStream_t s);

// plane.hip -- batched LiDAR ground-plane RANSAC
size_t mlg_plane_ws_bytes(int S, int H);
int mlg_plane_ransac_run(const float* pts, const int32_t* offs, int S, int H, uint64_t seed, double thr, void* ws,
                         size_t ws_bytes, double* plane, double* ratio, int32_t* inliers, hipStream_t s);
