/*
 * mlgate -- MI355X-native semantic loop-closure gate: public C ABI.
 *
 * The reference (wadewilliamsw1234/Multi-level-Indoor-SLAM) is pure Python; its hot
 * path is the class API of scripts/semantic_gating.  This library is the native
 * layer under the drop-in Python mirror (multi-level-indoor-slam_amd/mlgate), and
 * each entry point below names the reference method whose work it replaces.
 *
 * Conventions
 *   - every function returns int status: 0 ok, <0 error (MLG_E*); nothing throws;
 *   - all array arguments are DEVICE pointers (hipMalloc / torch CUDA tensors) unless
 *     documented otherwise, caller-allocated; `stream` is a hipStream_t (NULL = the
 *     default stream); every call is asynchronous on that stream;
 *   - bf16 buffers are raw uint16_t bit patterns (round-to-nearest-even);
 *   - no call allocates, frees or synchronises, so every call can be captured in a
 *     hipGraph; workspaces are sized by the *_workspace_bytes queries.
 */
#ifndef MLGATE_H
#define MLGATE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MLG_OK 0
#define MLG_EINVAL (-1)
#define MLG_EHIP (-2)
#define MLG_ENOMEM (-3)

#define MLG_VIT_DEPTH 12
#define MLG_VIT_EMBED 768
#define MLG_VIT_PATCH_K 768 /* 3*14*14 = 588 patch inputs, zero-padded to 12 K-tiles of 64 */

/* Struct arguments.  Every struct an entry point takes (mlg_vit_weights, mlg_salad_weights,
 * mlg_rn_weights, mlg_sp_weights, mlg_lg_weights, mlg_sg_weights, mlg_loftr_weights,
 * mlg_orb_params) begins with a head: struct_size = sizeof(the struct) and abi_version =
 * MLG_ABI_VERSION, both set by initialising it with MLG_STRUCT_INIT(type).  A struct whose
 * head disagrees -- built against another version of this header (a shorter or longer
 * struct), truncated, or not initialised -- is rejected with MLG_EINVAL (size queries
 * taking one return 0) before any field past the head is read.
 * Versions: 2 (round 5) appended mlg_vit_weights.packing and mlg_loftr_weights.coarse_tails;
 * 3 (round 6) added the heads. */
#define MLG_ABI_VERSION 3
#define MLG_STRUCT_INIT(T) {(uint32_t)sizeof(T), (uint32_t)MLG_ABI_VERSION}
int mlg_abi_version(void); /* MLG_ABI_VERSION of the library */
const char* mlg_strerror(int status);

/* ------------------------------------------------------------------ ViT-B/14 --
 * Device weights of the hub dinov2_vitb14 network in kernel layout (see
 * mlgate/vit.py:_pack_weights): GEMM weights bf16 [out, in] (nn.Linear layout),
 * everything else float32.  `pos` is the position embedding already resampled to
 * the (S/14)^2 patch grid (hub interpolate_pos_encoding), [1 + (S/14)^2, 768].
 */
typedef struct mlg_vit_block {
    const float *norm1_w, *norm1_b;
    const uint16_t* qkv_w; /* [2304, 768] */
    const float* qkv_b;
    const uint16_t* proj_w; /* [768, 768] */
    const float *proj_b, *ls1;
    const float *norm2_w, *norm2_b;
    const uint16_t* fc1_w; /* [3072, 768] */
    const float* fc1_b;
    const uint16_t* fc2_w; /* [768, 3072] */
    const float *fc2_b, *ls2;
} mlg_vit_block;

typedef struct mlg_vit_weights {
    uint32_t struct_size, abi_version; /* MLG_STRUCT_INIT(mlg_vit_weights) */
    const uint16_t* patch_w; /* [768, MLG_VIT_PATCH_K], k = c*196 + ky*14 + kx */
    const float* patch_b;
    const float* cls;        /* [768] */
    const float* pos;        /* [1 + P, 768] */
    mlg_vit_block blocks[MLG_VIT_DEPTH];
    const float *norm_w, *norm_b;
    int packing; /* 0: plain bf16 GEMM weights; MLG_VIT_SPLIT: [W_hi | W_lo] packing (must match the flag) */
} mlg_vit_weights;

/* mlg_vit_forward flags */
#define MLG_VIT_POOL_MEAN 1     /* AnyLoc: mean over patch tokens (place_recognition.py:485) instead of GeM */
#define MLG_VIT_KEEP_CHANNELS 2 /* AnyLoc._preprocess feeds 3-channel frames unswapped (:495-505) */
/* Split-bf16 ("precise") forward: every GEMM / attention operand x is carried as the
 * bf16 pair hi = bf16(x), lo = bf16(x - hi) (x = hi + lo to ~2^-17) and every product as
 * hi*hi + hi*lo + lo*hi with f32 accumulation (three MFMAs).  The GEMM weights must then
 * be packed [out, 2 * in] = [W_hi | W_lo] along the reduction dimension (the patch weight
 * [768, 2 * MLG_VIT_PATCH_K]) and mlg_vit_weights.packing set to MLG_VIT_SPLIT; a flag that
 * disagrees with the packing returns MLG_EINVAL.  Descriptor error against the fp32 network
 * drops from ~1e-5 to ~1e-11 (1 - cos), so kNN rankings follow the fp32 reference's to
 * its own near-tie level. */
#define MLG_VIT_SPLIT 4

/* Workspace for a batch of `batch` frames at network input size `image_size` (322).  The
 * size always covers the split forward (MLG_VIT_SPLIT): its [hi | lo] operand rows double
 * the bf16 activation buffers, so a plain-bf16 caller gets ~2x the operand memory it uses
 * (about 4.4 GB instead of ~2.4 GB at batch 246), in exchange for one size query for both. */
size_t mlg_vit_workspace_bytes(int batch, int image_size);

/*
 * CricaVPR descriptor path for a batch of frames, replacing, per frame,
 *   CricaVPR._preprocess            place_recognition.py:781-803
 *   backbone.get_intermediate_layers place_recognition.py:634 (hub DINOv2 forward)
 *   GeM pooling                      place_recognition.py:636-641
 *   extract_local_features           place_recognition.py:645-667 (same forward)
 * and, with flags = MLG_VIT_POOL_MEAN | MLG_VIT_KEEP_CHANNELS at image_size 518,
 * AnyLoc.extract_descriptor (place_recognition.py:467-505).
 * frames: uint8 [batch, H, W, C] (C = 1 gray, 3 BGR, 4 BGRA), frame_stride bytes
 * between frames.  desc_out: float32 [batch, 768].  local_out: float32
 * [batch, (S/14)^2 - 1, 768] or NULL.
 */
int mlg_vit_forward(const mlg_vit_weights* w, const uint8_t* frames, int batch, int H, int W, int C,
                    long frame_stride, int image_size, int flags, void* workspace, size_t workspace_bytes,
                    float* desc_out, float* local_out, void* stream);

/* ------------------------------------------------------------------- SALAD --
 * SALAD's native branch (place_recognition.py:357-368, 380-391): serizba/salad's
 * aggregator over the same DINOv2 ViT-B/14 (all final-LayerNorm tokens).  Weights in
 * kernel layout (mlgate/vpr.py SaladGPU._pack):
 *   w1 bf16 [1024, 768]  rows 0..511 cluster_features.0, 512..1023 score.0 (1x1 convs)
 *   w2 bf16 [256, 1024]  rows 0..127 [cluster_features.3 | 0], 128..191 [0 | score.3],
 *                        192..255 zero; b1 [1024], b2 [256] float32
 *   wt1 [512, 768], wt2 [256, 512] float32 token_features.0 / .2 (+ biases)
 *   dust_bin             the learned dust-bin score
 */
typedef struct mlg_salad_weights {
    uint32_t struct_size, abi_version; /* MLG_STRUCT_INIT(mlg_salad_weights) */
    const uint16_t* w1;
    const float* b1;
    const uint16_t* w2;
    const float* b2;
    const float *wt1, *bt1, *wt2, *bt2;
    float dust_bin;
} mlg_salad_weights;

#define MLG_SALAD_DIM 8448 /* 256 token + 64 clusters x 128 */

size_t mlg_salad_workspace_bytes(int batch, int image_size);

/*
 * SALAD descriptors for a batch of frames at image_size 322 (SALAD's evaluation size;
 * the hub PatchEmbed rejects the reference's 480 x 640 resize): preprocessing without a
 * channel swap, the ViT forward, the final LayerNorm over every token, then per frame
 * the token MLP, 3 log-domain Sinkhorn iterations over the [64 + dust-bin, 529] score
 * matrix, the cluster aggregation and the L2 normalisations.  desc_out float32
 * [batch, MLG_SALAD_DIM].
 */
int mlg_salad_forward(const mlg_vit_weights* w, const mlg_salad_weights* sw, const uint8_t* frames, int batch,
                      int H, int W, int C, long frame_stride, int image_size, void* workspace,
                      size_t workspace_bytes, float* desc_out, void* stream);

/* --------------------------------------------------------------- retrieval --
 * SemanticPlaceRecognition.find_loop_closures (place_recognition.py:851-911) for
 * query rows [q0, q0 + Q) against all N descriptors:
 *   normalise rows (bit-identical to the reference's numpy float32 norm + divide,
 *   place_recognition.py:186-187), S = Xn[q0:q0+Q] . Xn^T (float32), mask
 *   |t_j - t_i| < min_gap, top-k by (sim desc, index desc), drop sim < thr, floor bit.
 * desc: float32 [N, D]; t: float64 [N]; floor: int64 [N]; has_floor: uint8 [N]
 * (0 = floor_label None).  Outputs (device): idx int32 [Q, k], sim float32 [Q, k],
 * valid uint8 [Q, k], count int32 [Q] (entries per row, in emission order);
 * totals uint64[2] (+= valid, rejected) or NULL.  k >= 1, unbounded (k > 256: a per-row
 * radix select over (similarity, index) keys, in windows of 4096 ranks).
 */
size_t mlg_knn_workspace_bytes(int N, int D, int Q);
/* Workspace for a given k, for mlg_knn_gate (query = 0) or mlg_knn_query (query = 1):
 * for k <= 32 and D % 4 == 0 the scan is fused -- tiles of S stream through LDS into
 * per-row top-k lists, no [Q, N] matrix -- and needs only the normalised rows and
 * Q * splits * (8 k + 4) B of partial lists; otherwise = mlg_knn_workspace_bytes.
 * mlg_knn_workspace_bytes(N, D, Q) is always sufficient. */
size_t mlg_knn_workspace_bytes_k(int N, int D, int Q, int k, int query);
int mlg_knn_gate(const float* desc, int N, int D, const double* t, const int64_t* floor, const uint8_t* has_floor,
                 double min_gap, float thr, int k, int gating, int q0, int Q, void* workspace,
                 size_t workspace_bytes, int32_t* idx, float* sim, uint8_t* valid, int32_t* count,
                 unsigned long long* totals, void* stream);

/* BasePlaceRecognition.query (place_recognition.py:117-163) for Q query descriptors
 * against a database of N: cosine similarity, |t_db - t_query| < min_gap masked
 * (t_query NaN = no timestamp), top-k (no threshold).  Same workspace query. */
int mlg_knn_query(const float* db, int N, int D, const float* qdesc, int Q, const double* t_db,
                  const double* t_query, double min_gap, int k, void* workspace, size_t workspace_bytes,
                  int32_t* idx, float* sim, int32_t* count, void* stream);

/* Building blocks: compute_all_pairwise_similarities (place_recognition.py:179-190)
 * = row normalise (numpy-exact) + S[Q, N] = A . B^T in float32. */
int mlg_row_normalize_f32(const float* X, float* Xn, int N, int D, float* norms_or_null, void* stream);
int mlg_similarity(const float* A, int Q, const float* B, int N, int D, float* S, void* stream);

/* CricaVPR.compute_cross_correlation_score (place_recognition.py:669-712):
 * rows of q [n1, D] and m [n2, D] L2-normalised, C = q m^T, score (device float) =
 * sqrt(mean_i max_j C * mean_j max_i C). */
size_t mlg_xcorr_workspace_bytes(int n1, int n2, int D);
int mlg_xcorr_score(const float* q, int n1, const float* m, int n2, int D, void* workspace, size_t workspace_bytes,
                    float* score, void* stream);

/* CricaVPR.rerank_candidates at scale (place_recognition.py:714-757): the
 * compute_cross_correlation_score of P (query, candidate) pairs in one pass.  feats: f32
 * [F, L, D] local features of F frames (not normalised); query / cand: device int32 [P]
 * frame indices; scores: device f32 [P], each bit-identical to mlg_xcorr_score on that
 * pair (same row normalisation, same exact-f32 MFMA tiles, same reduction order); no
 * [L, L] matrix is written. */
size_t mlg_xcorr_batch_workspace_bytes(int F, int L, int D, int P);
int mlg_xcorr_batch(const float* feats, int F, int L, int D, const int32_t* query, const int32_t* cand, int P,
                    void* workspace, size_t workspace_bytes, float* scores, void* stream);

/* ----------------------------------------------------------- op-level access --
 * Individual kernels of the ViT path (parity tests against a float32 reference). */
int mlg_op_gemm_f32out(const uint16_t* A, const uint16_t* W, float* C, int M, int N, int K, void* stream);
/* GEMM kernel generation (all bit-identical): 1 = 128x128 register-staged;
 * 2 = 128x256 3-stage LDS-DMA, BK 64 (N % 256 == 0 and K / 64 % 3 == 0);
 * 3 = the same with BK 32 (K / 32 % 3 == 0); 4 = persistent 256x256 2-stage LDS-DMA,
 * one workgroup per CU walking XCD-local tiles (default; N % 256 == 0,
 * K / 64 even).  A shape a variant cannot take falls back 4 -> 2 -> 1. */
int mlg_set_gemm_variant(int variant);
int mlg_op_gemm_f32out_variant(int variant, const uint16_t* A, const uint16_t* W, float* C, int M, int N, int K,
                               void* stream);
int mlg_op_gemm_bias_gelu(const uint16_t* A, const uint16_t* W, const float* bias, uint16_t* C, int M, int N,
                          int K, void* stream);
int mlg_op_gemm_residual(const uint16_t* A, const uint16_t* W, const float* bias, const float* gamma, float* X,
                         int M, int N, int K, void* stream);
int mlg_op_layernorm_bf16(const float* X, const float* g, const float* b, uint16_t* Y, int M, void* stream);
/* ViT attention (hub Attention.forward, 12 heads x 64) on the pipelined tile: Q, K bf16
 * [12][B * Tpad][64], Vt bf16 [12][B * Tpad / 64][64 d][64 keys] (keys >= T finite), O bf16
 * [B * T][768]; task_ws: 5 * B int32 of device scratch. */
int mlg_op_attention(const uint16_t* Q, const uint16_t* K, const uint16_t* Vt, uint16_t* O, int B, int T, int Tpad,
                     int32_t* task_ws, void* stream);
/* Ragged multi-head attention (LightGlue self / cross, geometric_verification.py:263-312
 * via upstream SelfBlock / CrossBlock).  Task t = int32 x4 (q_off, q_len, kv_off, kv_len)
 * over a flat token layout; Q, K bf16 [heads][Npad][64] (Q pre-scaled by 1/8 is NOT
 * assumed: the kernel scales), Vt bf16 tiled [heads][Npad/64][64 d][64 keys]; output row
 * out_off[t] + r of O [Npad][ldo] at column h*64.  Device pointers. */
int mlg_op_attention_varlen(const uint16_t* Q, const uint16_t* K, const uint16_t* Vt, uint16_t* O, int ldo, int Npad,
                            int heads, const int32_t* tasks, const int32_t* out_off, int ntasks, int max_q,
                            void* stream);
/* Fused LightGlue block tail (SelfBlock / CrossBlock after the attention):
 * msg = ctx Wout^T + bout; X += Wf2 GELU(LN(Wf1 [bf16(X) | bf16(msg)] + bf1)) + bf2 for M token
 * rows; X f32 [M][256] in place; xcopy [M][ldc] cols 0..255 holds bf16(X) on entry (the
 * GEMM operand, as the previous block left it) and on exit.  bf16 weights
 * packed k-step-major: W[n][k] of an nn.Linear ([out][in]) stored at [k/16][n][k%16].
 * Device pointers. */
int mlg_op_lg_ffn(const uint16_t* ctx, float* X, uint16_t* xcopy, int ldc, int M, const uint16_t* Wout,
                  const float* bout, const uint16_t* Wf1, const float* bf1, const float* ln_g, const float* ln_b,
                  const uint16_t* Wf2, const float* bf2, void* stream);
/* LightGlue block projections (lg_proj.hip): self_block != 0: q, k, v = Wqkv x + b with
 * rotary on q and k; else qk = to_qk x, v = to_v x.  The rotary factors come interleaved in
 * `ecos`, f32 [Npad / 64][16][64][4]: for token row r and frequency pair p the four floats
 * (cos 2p, cos 2p + 1, sin 2p, sin 2p + 1) at ((r / 64) * 16 + p) * 64 + r % 64 (round 5:
 * one conflict-free 16-B LDS read per lane; mlgate.lightglue.pack_rotary); `esin` is
 * unused (NULL).  xcopy
 * bf16 [Npad][ldx] (cols 0..255), W k-step-major [16][768 | 512][16] with rows
 * [q|k|v] x (head, 64) (self) or [qk | v]; outputs Q, K bf16 [4][Npad][64], Vt bf16
 * [4][Npad/64][64][64]; rows with live[m] == 0 written as zeros.  Npad % 64 == 0. */
int mlg_op_lg_proj(int self_block, const uint16_t* xcopy, int ldx, const uint16_t* W, const float* bias,
                   const float* ecos, const float* esin, const uint8_t* live, uint16_t* Q, uint16_t* K, uint16_t* Vt,
                   int Npad, void* stream);
/* Implicit-GEMM convolution of LoFTR's ResNetFPN (loftr.hip convs): k x k (k = 1 or 3,
 * zero padding k / 2) stride-s conv of NHWC bf16 in [B, H, W, C] (C % 64 == 0) with
 * weights bf16 [N][k * k * C] (k index tap * C + c, N % 128 == 0) plus bias -> f32 out
 * [B, Ho, Wo, N], Ho = ceil(H / s); zero16 = 16 zero bytes on the device. */
int mlg_op_conv2d_nhwc(const uint16_t* in, const uint16_t* zero16, int B, int H, int W, int C, int k, int s,
                       const uint16_t* Wt, const float* bias, float* out, int N, void* stream);
int mlg_op_preprocess_patches(const uint8_t* frames, int B, int H, int W, int C, long frame_stride, int S,
                              uint16_t* patches, void* stream);

/* ----------------------------------------------- LiDAR ground plane --
 * Replaces LiDARFloorTracker.fit_ground_plane_ransac (lidar_floor_tracker.py:92-141)
 * for S scans at once: scan s owns ground points [offsets[s], offsets[s+1]) of pts
 * (device f32 [N, 3]).  `iterations` 3-point hypotheses per scan (counter-based RNG of
 * (seed, hypothesis)); inlier iff |n . p + d| < threshold (float64); best = most
 * inliers, first on ties.  Outputs (device): plane f64 [S, 4] (NaN if none), inlier
 * ratio f64 [S], inlier count int32 [S]. */
size_t mlg_plane_ransac_workspace_bytes(int S, int iterations);
int mlg_plane_ransac(const float* pts, const int32_t* offsets, int S, int iterations, uint64_t seed, double threshold,
                     void* workspace, size_t workspace_bytes, double* plane, double* ratio, int32_t* inliers,
                     void* stream);

/* ------------------------------------------------- trajectory proximity --
 * Replaces detect_loop_closure_candidates + apply_floor_gating of the SLAM
 * integrations (scripts/semantic_gating/orb_slam3_integration.py:167-281,
 * lego_loam_integration.py:121-204): every pair (i, j), j - i >= min_gap,
 * ||p_i - p_j|| <= radius (float64, inclusive), for query rows i in
 * [row0, row0 + nrows), emitted in (i, j) order with the float64 distance and the
 * SemanticLoopClosureGate verdict (strict: equal floors; non-strict: |diff| <= 1).
 * pos: device float64 [N, 3]; floor: device int64 [N] or NULL (all accepted).
 * Two calls share one workspace: mlg_proximity_count writes the device int64
 * totals[2] = {candidates, accepted}; the caller sizes the outputs from totals[0]
 * and calls mlg_proximity_emit with the same arguments.  N <= 65536. */
size_t mlg_proximity_workspace_bytes(int N, int nrows);
int mlg_proximity_count(const double* pos, const int64_t* floor, int N, int row0, int nrows, double radius,
                        int min_gap, int strict, void* workspace, size_t workspace_bytes, long long* totals,
                        void* stream);
int mlg_proximity_emit(const double* pos, const int64_t* floor, int N, int row0, int nrows, double radius,
                       int min_gap, int strict, const void* workspace, size_t workspace_bytes, int32_t* pairs,
                       double* dist, uint8_t* valid, void* stream);

/* ----------------------------------------------------------- ResNet-50 --
 * Replaces MixVPR / SALAD's executed path, the torchvision ResNet-50 fallback
 * (scripts/semantic_gating/place_recognition.py:248-306): BGR taken as RGB ->
 * Pillow bilinear (antialiased) resize to 224x224 -> /255 -> ImageNet normalise ->
 * resnet50 minus fc -> 2048-d global average pool, zero-padded / truncated to
 * descriptor_dim.  BatchNorm (eval) folded into the conv weights / biases by the
 * caller.  frames: device uint8 [B] x (H x W x C), C in {1, 3, 4}; desc: device f32
 * [B, descriptor_dim]. */
typedef struct mlg_rn_block {
    const uint16_t* w1; const float* b1;  /* conv1 1x1: bf16 [max(width,128)][Cin] (rows >= width zero) */
    const uint16_t* w2; const float* b2;  /* conv2 3x3: bf16 [max(width,128)][9 * width], k = tap * width + c */
    const uint16_t* w3; const float* b3;  /* conv3 1x1: bf16 [4 width][width] */
    const uint16_t* wd; const float* bd;  /* downsample 1x1: bf16 [4 width][Cin], or NULL */
} mlg_rn_block;
typedef struct mlg_rn_weights {
    uint32_t struct_size, abi_version; /* MLG_STRUCT_INIT(mlg_rn_weights) */
    const float* stem_w;  /* f32 [64][7][7][3] */
    const float* stem_b;  /* f32 [64] */
    mlg_rn_block blocks[16];
} mlg_rn_weights;
size_t mlg_resnet50_workspace_bytes(int B, int H, int W);
int mlg_resnet50_forward(const mlg_rn_weights* w, const uint8_t* frames, int B, int H, int W, int C,
                         long frame_stride, int descriptor_dim, void* workspace, size_t workspace_bytes,
                         float* desc, void* stream);
/* Parity entry: only the Pillow bilinear resize of the above -> uint8 [B, 224, 224, 3]
 * (workspace sized by mlg_resnet50_workspace_bytes). */
int mlg_op_pillow_resize_224(const uint8_t* frames, int B, int H, int W, int C, long frame_stride, void* workspace,
                             size_t workspace_bytes, uint8_t* out, void* stream);

/* -------------------------------------------------------- SuperPoint --
 * Replaces the extractor half of LightGlue._detect_and_match_native
 * (scripts/semantic_gating/geometric_verification.py:263-312): cv2 BGR2GRAY / 255 ->
 * LightGlue's SuperPoint(max_num_keypoints, detection_threshold) forward (NMS radius,
 * border removal, top-k, bilinear descriptor sampling) for B frames at once.
 * frames: device uint8 [B] x (H x W x C), C in {1, 3 (BGR), 4}, H, W >= 16 (the score
 * map and keypoints cover 8 floor(H/8) x 8 floor(W/8) after the encoder's round-down pools).
 * Outputs (device): keypoints f32 [B, max_kp, 2] (x, y), scores f32 [B, max_kp],
 * descriptors f32 [B, max_kp, 256] (unit L2; zero rows past counts[b]) and optionally
 * the same in bf16, counts int32 [B].  Keypoint order: raster order when at most
 * max_kp pass the threshold, else score-descending (raster index ascending on ties). */
typedef struct mlg_sp_weights {
    uint32_t struct_size, abi_version; /* MLG_STRUCT_INIT(mlg_sp_weights) */
    const float* conv1a_w;  /* f32 [64][3][3] */
    const float* conv1a_b;  /* f32 [64] */
    const uint16_t* w[11];  /* bf16: conv1b conv2a conv2b conv3a conv3b conv4a conv4b convPa
                               ([Cout][3][3][Cin]); convPb [128][256] (rows 65..127 zero);
                               convDa [256][3][3][128]; convDb [256][256] */
    const float* b[11];     /* f32 [Cout] */
} mlg_sp_weights;
size_t mlg_superpoint_workspace_bytes(int B, int H, int W);
int mlg_superpoint(const mlg_sp_weights* w, const uint8_t* frames, int B, int H, int W, int C, long frame_stride,
                   float detection_threshold, int max_keypoints, int nms_radius, int remove_borders, void* workspace,
                   size_t workspace_bytes, float* keypoints, float* scores, float* descriptors,
                   uint16_t* descriptors_bf16, int32_t* counts, void* stream);

/* --------------------------------------------------------- LightGlue --
 * Replaces the matcher half of LightGlue._detect_and_match_native
 * (geometric_verification.py:263-312): LightGlue(features='superpoint') defaults --
 * 9 layers, 4 heads, d 256, depth_confidence 0.95, width_confidence 0.99,
 * filter_threshold 0.1, point pruning while a side has more than `pruning_min_kpts`
 * tokens (1536 on CUDA with flash) -- for P pairs at once.  Features of F frames
 * (e.g. mlg_superpoint outputs): keypoints f32 [F, kmax, 2], descriptors f32
 * [F, kmax, 256] on the device, counts [F] on the HOST; pair p matches frame
 * pair_a[p] (image0) against pair_b[p] (image1), both HOST arrays.  Outputs (device):
 * matches int32 [P, kmax, 2] (indices into the two frames' keypoints, ascending in the
 * image0 index), scores f32 [P, kmax] (the reference's matching scores), num_matches
 * int32 [P]; stop_layer (host, optional): layers run per pair.  Synchronises `stream`
 * once per layer (early-stop / pruning decisions). */
typedef struct mlg_lg_block {
    const uint16_t* Wqkv; const float* bqkv;  /* self: Wqkv [768][256] (rows as [q|k|v] x (head, 64));
                                                 cross: [to_qk; to_v] [512][256]; k-step-major */
    const uint16_t* Wout; const float* bout;  /* out_proj / to_out [256][256]  } k-step-major: */
    const uint16_t* Wf1;  const float* bf1;   /* ffn.0 [512][512]             } W[n][k] at   */
    const float* ln_g;    const float* ln_b;  /* ffn.1 LayerNorm(512)                          */
    const uint16_t* Wf2;  const float* bf2;   /* ffn.3 [256][512]             } [k/16][n][k%16] */
} mlg_lg_block;
typedef struct mlg_lg_weights {
    uint32_t struct_size, abi_version;                     /* MLG_STRUCT_INIT(mlg_lg_weights) */
    const float* Wr;                                       /* posenc.Wr [32][2] f32 */
    mlg_lg_block self[9], cross[9];                        /* bf16 weights, f32 biases */
    const uint16_t* Wfinal[9]; const float* bfinal[9];     /* log_assignment.i.final_proj */
    const float* wmatch[9];    const float* bmatch[9];     /* log_assignment.i.matchability */
    const float* wconf[8];     const float* bconf[8];      /* token_confidence.i.token.0 */
    const float* ones;                                     /* f32 [256] of 1.0 */
} mlg_lg_weights;
size_t mlg_lightglue_workspace_bytes(int P, int kmax);
int mlg_lightglue(const mlg_lg_weights* w, const float* keypoints, const float* descriptors, const int32_t* counts,
                  int F, int kmax, const int32_t* pair_a, const int32_t* pair_b, int P, float depth_confidence,
                  float width_confidence, float filter_threshold, int pruning_min_kpts, void* workspace,
                  size_t workspace_bytes, int32_t* matches, float* scores, int32_t* num_matches, int32_t* stop_layer,
                  void* stream);

/* LightGlue is symmetric in its two images (shared weights; self / cross blocks, the
 * dual-softmax assignment, early stopping and pruning all treat image0 and image1 alike),
 * so the full gate matches each unordered pair once.  This gathers, per ordered pair p,
 * the matches of unordered row rows[p] of a mlg_lightglue output; with swap[p] != 0 the
 * image roles are exchanged and the matches re-sorted ascending in the new image0 index
 * -- the order the swapped call returns.  matches_out int32 [P, kmax, 2], scores_out
 * f32 [P, kmax], num_out int32 [P]; rows / swap device arrays. */
int mlg_lg_orient_matches(const int32_t* matches, const float* scores, const int32_t* num_matches,
                          const int32_t* rows, const uint8_t* swap, int P, int kmax, int32_t* matches_out,
                          float* scores_out, int32_t* num_out, void* stream);

/* Diagnostics (tools/lg_determinism.py; no reference counterpart): between _begin and
 * _end, the CALLING THREAD's mlg_lightglue calls append, after every stage, one 64-bit
 * hash per 64-row tile of the buffer the stage wrote into dev_buf (uint64 words, device
 * memory).  _end returns the number of stages recorded (tags[i] = layer * 100 + stage,
 * layer 99 = layer 0's per-frame self block; counts[i] = its hashes, in buffer order)
 * or MLG_ENOMEM if dev_buf was too small. */
int mlg_dbg_lg_trace_begin(void* dev_buf, size_t bytes);
int mlg_dbg_lg_trace_end(int32_t* tags, int32_t* counts, int max_entries);
/* Diagnostics (tools/ffn_interference.py): fill every CU's 160 KiB of LDS (sink: a device
 * int32 [256] scratch that is never written for patterns other than 0x12345679), or every
 * SIMD's 512 VGPRs + AGPRs, with `pattern` -- a kernel launched next on `stream` that
 * reads LDS or registers it never wrote then shows pattern-dependent results. */
int mlg_dbg_fill_lds(uint32_t pattern, void* sink, void* stream);
int mlg_dbg_fill_regs(uint32_t pattern, void* stream);
/* Diagnostics (tests/test_ransac_gpu.py): while `on`, every mlg_ransac_epipolar call of
 * this process overwrites the solution count of each hypothesis slot no pair uses (h > 0
 * of a 5 / 7-point direct pair, h >= the subset count of a RANSAC pair, every slot of a
 * pair without a model) with `value` after the solvers ran -- a stand-in for a solver that
 * leaves a slot unwritten; the readers clamp counts to [0, 10], so results must not change. */
int mlg_dbg_ransac_poison_nsol(int on, int value);
/* Diagnostics (tools/ffn_trace.py): in a build with -DMLG_FFN_TRACE=1, copies the phase
 * timestamps of the last fused-block-tail launch (per workgroup: 10 s_memtime values, the
 * wave's HW_ID and XCC_ID; [65536][12] uint64) to host memory; MLG_EINVAL in the product. */
int mlg_dbg_ffn_trace(void* host, size_t bytes);
/* Diagnostics (tools/attn_trace.py): in a build with -DMLG_ATT_TRACE=1, the phase stamps of
 * the last LightGlue attention launch (per logical workgroup: entry, prologue done, stage
 * loop done, end, HW_ID, XCC_ID, query count, written flag; [65536][8] uint64); MLG_EINVAL
 * in the product. */
int mlg_dbg_att_trace(void* host, size_t bytes);

/* --------------------------------------------------------- SuperGlue --
 * The SuperGlue matcher of the reference's SuperGlue class configuration
 * (geometric_verification.py:385-399: weights 'indoor', sinkhorn_iterations 20,
 * match_threshold 0.2), whose native branch the reference never reaches (:419-421):
 * keypoint encoder, 18-layer attentional GNN, final_proj, log-space optimal transport
 * with the learned dustbin score, mutual-nearest matches above the threshold.
 * Features as mlg_lightglue plus keypoint scores f32 [F, kmax]; W, H the frame size
 * (keypoint normalisation).  layer[l] reuses the LightGlue block table: Wqkv = the three
 * attention projections (rows permuted so each head's 64 channels are contiguous:
 * SuperGlue's view(b, 64, 4, n) interleaves them), Wout = merge (input columns permuted
 * the same way), Wf1 / bf1 = mlp.0 with mlp.1 BatchNorm folded, ln_g / ln_b unused,
 * Wf2 / bf2 = mlp.3.  kenc_w[0..2] f32 [out][in] (BN folded), kenc_w4 / kenc_w5 and
 * Wfinal bf16 [out][in] (not k-step-major).  Outputs as mlg_lightglue (matches
 * ascending in the image0 index).  Synchronises `stream`. */
typedef struct mlg_sg_weights {
    uint32_t struct_size, abi_version; /* MLG_STRUCT_INIT(mlg_sg_weights) */
    const float* kenc_w[3]; const float* kenc_b[3];
    const uint16_t* kenc_w4; const float* kenc_b4;
    const uint16_t* kenc_w5; const float* kenc_b5;
    mlg_lg_block layer[18];
    const uint16_t* Wfinal; const float* bfinal;
    float bin_score;
} mlg_sg_weights;
size_t mlg_superglue_workspace_bytes(int P, int kmax);
int mlg_superglue(const mlg_sg_weights* w, const float* keypoints, const float* scores, const float* descriptors,
                  const int32_t* counts, int F, int kmax, int W, int H, const int32_t* pair_a, const int32_t* pair_b,
                  int P, int sinkhorn_iterations, float match_threshold, void* workspace, size_t workspace_bytes,
                  int32_t* matches, float* match_scores, int32_t* num_matches, void* stream);

/* ------------------------------------------------------------ RANSAC --
 * Batched replacement for BaseFeatureMatcher.verify_geometric_consistency and
 * estimate_relative_pose (scripts/semantic_gating/geometric_verification.py:104-188),
 * i.e. cv2.findEssentialMat(RANSAC, prob 0.999) / cv2.findFundamentalMat(FM_RANSAC)
 * and cv2.recoverPose, for P pairs at once.  Pair p owns matches
 * [offsets[p], offsets[p+1]) of kp1 / kp2 (device float32 [S_total, 2], pixels).
 * K: device float64 3x3 row-major per pair (k_stride 9) or shared (k_stride 0), or
 * NULL for the fundamental-matrix path.  `hypotheses` minimal samples per pair
 * (5-point for E, 7-point for F) are drawn from a counter-based RNG (`seed`),
 * solved and scored in parallel; the best model has the most inliers (lowest
 * hypothesis index on ties).  Outputs (device): model float64 [P, 9] (E or F),
 * mask uint8 [S_total], inliers int32 [P], pose float64 [P, 16] ([R|t; 0 0 0 1],
 * may be NULL; E path only), status int32 [P]: 0 ok, 1 no model (E: < 5 matches;
 * F: < 7), 2 model but fewer than 5 inliers (no pose). */
size_t mlg_ransac_workspace_bytes(int P, long S_total, int hypotheses);
int mlg_ransac_epipolar(const float* kp1, const float* kp2, const int32_t* offsets, int P, long S_total,
                        const double* K, int k_stride, double threshold, int hypotheses, uint64_t seed,
                        void* workspace, size_t workspace_bytes, double* model, uint8_t* mask, int32_t* inliers,
                        double* pose, int32_t* status, void* stream);
/* cv2.recoverPose(E, k1[mask], k2[mask], K) for P pairs given E [P, 9] and mask
 * (geometric_verification.py:155-188): pose [P, 16]; zeros when < 5 inliers. */
int mlg_recover_pose(const float* kp1, const float* kp2, const int32_t* offsets, int P, const double* K,
                     int k_stride, const double* E, const uint8_t* mask, double* pose, void* stream);

/* ------------------------------------------------------------------ LoFTR --
 * Replaces LoFTR.detect_and_match (geometric_verification.py:458-526):
 * kornia.feature.LoFTR(pretrained='indoor') on cv2 BGR2GRAY / 255 frames whose H and W
 * are multiples of 8.  Weights are device pointers prepared on the host
 * (mlgate/loftr.py): eval BatchNorm folded into the convs, the 196-channel stages
 * zero-padded to 256, conv weights bf16 [Cout][k * k * Cin] with k index = tap * Cin + c.
 * conv_w order: layer1.{0,1}.conv{1,2} (0-3); layer2.0.conv1, .conv2, .downsample,
 * layer2.1.conv1, .conv2 (4-8); the same for layer3 (9-13); layer3_outconv,
 * layer2_outconv, layer2_outconv2.0 (+BN), layer2_outconv2.3 (14-17); layer1_outconv,
 * layer1_outconv2.0 (+BN), layer1_outconv2.3 (18-20).  conv_b: folded BN bias or NULL. */
#define MLG_LOFTR_NCONV 21
typedef struct {
    const uint16_t* w;      /* [3d][d] rows q | k | v (no bias) */
    const uint16_t* wmerge; /* [d][d] */
    const uint16_t* w1;     /* mlp.0 [2d][2d] */
    const uint16_t* w2;     /* mlp.2 [d][2d] */
    const float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
} mlg_loftr_layer;
typedef struct mlg_loftr_weights {
    uint32_t struct_size, abi_version; /* MLG_STRUCT_INIT(mlg_loftr_weights) */
    const float* stem_w; /* conv1 7x7 (BN folded) f32 [49][128] */
    const float* stem_b; /* [128] */
    const uint16_t* conv_w[MLG_LOFTR_NCONV];
    const float* conv_b[MLG_LOFTR_NCONV];
    mlg_loftr_layer coarse[8]; /* d 256, self / cross alternating */
    mlg_loftr_layer fine[2];   /* d 128 */
    const uint16_t* down_w;    /* fine_preprocess.down_proj [128][256] */
    const float* down_b;
    const uint16_t* merge_wf;  /* merge_feat weight columns 0..127 (window features) [128][128] */
    const uint16_t* merge_wc;  /* merge_feat weight columns 128..255 (coarse context) [128][128] */
    const float* merge_b;
    /* optional: the coarse layers' block-tail weights in the fused kernel's layout, written
     * once by mlg_loftr_pack_tails (mlg_loftr_tails_bytes() bytes of device memory); NULL:
     * mlg_loftr_match repacks them into its workspace on every call.  The pack is a COPY:
     * redo it whenever the coarse layers' merge / MLP / LayerNorm weights change, or the
     * fused tail keeps the old ones while the attention reads the new */
    const void* coarse_tails;
} mlg_loftr_weights;
size_t mlg_loftr_tails_bytes(void);
int mlg_loftr_pack_tails(const mlg_loftr_weights* w, void* out, void* stream);
/* Op-level check (tests/test_loftr_gpu.py): one coarse encoder layer (even: self on both
 * sides; odd: cross, side 0 then side 1) over x f32 [2 nseg L, 256] and cat bf16
 * [2 nseg L, 512] (cat[:, :256] = bf16(x)), in place; fused != 0 runs the block tail as
 * the one fused kernel the product uses, 0 as the unfused GEMM + LayerNorm sequence. */
size_t mlg_op_loftr_coarse_layer_ws_bytes(int nseg, int L);
int mlg_op_loftr_coarse_layer(const mlg_loftr_weights* w, int layer, int fused, float* x, uint16_t* cat, int nseg,
                              int L, void* workspace, size_t workspace_bytes, void* stream);
/* Backbone for B frames uint8 [B, H, W, C] (C = 3 BGR, 4 BGRA or 1 gray; frame_stride
 * bytes), H, W >= 32.  With H8 = H / 8 * 8, W8 = W / 8 * 8 (frames whose H or W is not a
 * multiple of 8 are converted and resized as the reference does: cv2 BGR2GRAY, then
 * cv2.resize INTER_LINEAR to W8 x H8): coarse f32 [B, H8/8 * W8/8, 256] (1/8 map,
 * row-major cells) and fine f32 [B, H8/2 * W8/2, 128]. */
size_t mlg_loftr_features_ws_bytes(int B, int H, int W);
int mlg_loftr_features(const mlg_loftr_weights* w, const uint8_t* frames, int B, int H, int W, int C,
                       long frame_stride, void* workspace, size_t workspace_bytes, float* coarse, float* fine,
                       void* stream);
/* Matching of P pairs (frames pa[p], pb[p]: HOST int32 arrays indexing coarse / fine;
 * H, W: the multiples of 8 the features were computed at; keypoints in that frame):
 * coarse transformer, dual-softmax coarse matches (conf > 0.2, 2-cell border, mutual
 * nearest), fine refinement.  pe: position encoding f32 [H/8 * W/8, 256] (device).
 * Outputs (device): counts int32 [P]; for pair p, match k < counts[p] (row order of the
 * coarse cell in frame pa[p]): kpts0 / kpts1 f32 [P, L, 2] at [p * L + k], conf f32
 * [P, L] (L = H/8 * W/8).  Synchronises the stream (the fine stage is sized by the
 * coarse counts).  Workspace (mlg_loftr_match_ws_bytes): the coarse transformer's token
 * buffers (~13 KB per token, 2 P L tokens: q / k / v f32 is the largest, and holds the
 * similarity's split-bf16 operand rows afterwards), the similarity of min(P, 8) pairs at a
 * time (L x roundup4(L) f32 each: 92 MB at 640 x 480, 145 MB at 720 x 536), and the fine
 * stage's buffers for 4096 matches at a time. */
size_t mlg_loftr_match_ws_bytes(int P, int H, int W);
/* The coarse similarity's arithmetic for the following mlg_loftr_match calls of this
 * process: exact = 0 (default) the split-bf16 product (hi*hi + hi*lo + lo*hi of the bf16
 * halves, f32 accumulation, ~6x the exact-f32 MFMA's rate; any frame size, the rows of S
 * padded to a multiple of 4 floats), exact = 1 the exact-f32 MFMA (A/B and parity tests:
 * tests/test_loftr_gpu.py compares the two arms pair by pair). */
int mlg_set_loftr_similarity(int exact);
int mlg_loftr_match(const mlg_loftr_weights* w, const float* coarse, const float* fine, int H, int W,
                    const int32_t* pa, const int32_t* pb, int P, const float* pe, void* workspace,
                    size_t workspace_bytes, int32_t* counts, float* kpts0, float* kpts1, float* conf, void* stream);

/* ------------------------------------------------------------- profiling --
 * Per-launch HIP-event timing of selected kernels, recorded on the stream the kernel
 * is launched on, with the algorithmic work of each launch (FLOPs; HBM bytes for slot
 * 8).  slot: 0 ViT fc1 GEMM, 1 fc2, 2 qkv, 3 proj, 4 ViT attention, 5 LightGlue
 * attention (ragged, all tasks of a launch), 6 LightGlue q/k/v projection GEMMs,
 * 7 SuperPoint 3x3 convs, 8 LightGlue fused block tail (out_proj + FFN).  slot_mask
 * selects the slots recorded (0 = off); a pool of 16384 event pairs is recycled by
 * mlg_prof_read / mlg_prof_read_work / mlg_prof_reset, which synchronise the recorded
 * events.  Not for use inside graph capture. */
int mlg_prof_enable(int slot_mask);
int mlg_prof_reset(void);
int mlg_prof_read(int slot, double* total_ms, long* launches);
int mlg_prof_read_work(int slot, double* flops);


/* ------------------------------------------------------ ORB + BFMatcher fallback --
 * LightGlue._load_fallback / _detect_and_match_fallback (geometric_verification.py:
 * 244-248, 314-350): cv2.ORB_create(nfeatures).detectAndCompute on BGR2GRAY frames and
 * cv2.BFMatcher(NORM_HAMMING, crossCheck=True).match sorted by distance, for a batch of
 * frames / pairs.  The ORB geometry (OpenCV ORB_Impl defaults: 8 levels x 1.2, edge 31,
 * FAST threshold 20, patch 31) is computed by the caller (mlgate/orb.py) into a HOST
 * mlg_orb_params; `pattern` is a device int16 [256 pairs][2 points][x, y] point table
 * (OpenCV's bit_pattern_31_ or, by default, its makeRandomPattern(31) stream).
 * Outputs per frame f, slots [f * max_kp, f * max_kp + counts[f]): keypoints (x, y) in
 * level-0 pixels, Harris responses, angles (degrees), levels, 32-byte descriptors, in
 * level order and within a level by (response desc, y, x).  counts[f] < 0: a per-level
 * candidate list overflowed (not expected below 16 M-pixel frames).
 */
#define MLG_ORB_LEVELS 8
typedef struct mlg_orb_params {
    uint32_t struct_size, abi_version; /* MLG_STRUCT_INIT(mlg_orb_params) */
    int level_w[MLG_ORB_LEVELS], level_h[MLG_ORB_LEVELS];
    int level_features[MLG_ORB_LEVELS]; /* nfeaturesPerLevel */
    float level_scale[MLG_ORB_LEVELS];
    int umax[16];
    float gauss[7]; /* getGaussianKernel(7, 2, CV_32F) of the per-level GaussianBlur */
    int fast_threshold, edge_threshold;
} mlg_orb_params;
size_t mlg_orb_workspace_bytes(const mlg_orb_params* p, int F, int H, int W, int max_kp);
int mlg_orb_detect(const mlg_orb_params* p, const int16_t* pattern, const uint8_t* frames, long frame_stride, int F,
                   int H, int W, int C, int max_kp, void* ws, size_t ws_bytes, float* keypoints, float* responses,
                   float* angles, int32_t* levels, uint8_t* descriptors, int32_t* counts, void* stream);
/* Cross-checked nearest neighbours of frames pair_a[p] -> pair_b[p] (descriptors /
 * counts as mlg_orb_detect wrote them), sorted by distance, ties by query index:
 * slots [p * max_kp, p * max_kp + nmatch[p]) of query_idx / train_idx / distance. */
size_t mlg_orb_match_workspace_bytes(int P, int max_kp);
int mlg_orb_match(const uint8_t* descriptors, const int32_t* counts, int max_kp, const int32_t* pair_a,
                  const int32_t* pair_b, int P, void* ws, size_t ws_bytes, int32_t* query_idx, int32_t* train_idx,
                  int32_t* distance, int32_t* nmatch, void* stream);

/* ---------------------------------------------------------- keyframe ingestion --
 * HOST pointers (not device): PNG keyframes -> BGR uint8 [n, H, W, 3], replacing the
 * cv2.imread(path) of process_image_sequence (place_recognition.py:965-968) on the
 * '{timestamp:.6f}.png' files scripts/utils/bag_utils.py:222-271 writes.  IMREAD_COLOR
 * semantics: palette -> RGB, gray -> 3 equal channels (1/2/4-bit samples scaled to
 * 0..255), alpha stripped, 16-bit samples -> high byte, Adam7 undone, stored as BGR.
 * A pool of `threads` host threads decodes image i into out + i*H*W*3 (pass a pinned
 * buffer and copy it to HBM on a side stream); status[i] = 0, MLG_EINVAL (unreadable,
 * corrupt or not a PNG: imread's None) or MLG_ESIZE (a valid PNG that is not H x W).
 */
#define MLG_ESIZE (-4)
int mlg_png_info(const uint8_t* data, size_t len, int32_t* width, int32_t* height, int32_t* color_type,
                 int32_t* bit_depth);
int mlg_png_decode_bgr(const uint8_t* const* data, const size_t* lens, int n, uint8_t* out, int H, int W,
                       int threads, int32_t* status);
int mlg_png_load_bgr(const char* const* paths, int n, uint8_t* out, int H, int W, int threads, int32_t* status);

#ifdef __cplusplus
}
#endif
#endif /* MLGATE_H */
