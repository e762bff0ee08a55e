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

int mlg_abi_version(void);
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
    const uint16_t* patch_w; /* [768, MLG_VIT_PATCH_K], k = c*196 + ky*14 + kx */
    const float* patch_b;
    const float* cls;        /* [768] */
    const float* pos;        /* [1 + P, 768] */
    mlg_vit_block blocks[MLG_VIT_DEPTH];
    const float *norm_w, *norm_b;
} mlg_vit_weights;

/* mlg_vit_forward flags */
#define MLG_VIT_POOL_MEAN 1     /* AnyLoc: mean over patch tokens (place_recognition.py:485) instead of GeM */
#define MLG_VIT_KEEP_CHANNELS 2 /* AnyLoc._preprocess feeds 3-channel frames unswapped (:495-505) */

/* Workspace for a batch of `batch` frames at network input size `image_size` (322). */
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

/* --------------------------------------------------------------- retrieval --
 * SemanticPlaceRecognition.find_loop_closures (place_recognition.py:851-911) for
 * query rows [q0, q0 + Q) against all N descriptors:
 *   normalise rows (bit-identical to the reference's numpy float32 norm + divide,
 *   place_recognition.py:186-187), S = Xn[q0:q0+Q] . Xn^T (float32), mask
 *   |t_j - t_i| < min_gap, top-k by (sim desc, index desc), drop sim < thr, floor bit.
 * desc: float32 [N, D]; t: float64 [N]; floor: int64 [N]; has_floor: uint8 [N]
 * (0 = floor_label None).  Outputs (device): idx int32 [Q, k], sim float32 [Q, k],
 * valid uint8 [Q, k], count int32 [Q] (entries per row, in emission order);
 * totals uint64[2] (+= valid, rejected) or NULL.  1 <= k <= 256.
 */
size_t mlg_knn_workspace_bytes(int N, int D, int Q);
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
int mlg_op_attention(const uint16_t* Q, const uint16_t* K, const uint16_t* Vt, uint16_t* O, int B, int T, int Tpad,
                     void* stream);
int mlg_op_preprocess_patches(const uint8_t* frames, int B, int H, int W, int C, long frame_stride, int S,
                              uint16_t* patches, void* stream);

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

/* ------------------------------------------------------------- profiling --
 * Per-launch HIP-event timing of selected kernels inside mlg_vit_forward, recorded on
 * the stream the kernel is launched on.  slot: 0 fc1 GEMM, 1 fc2 GEMM, 2 qkv GEMM,
 * 3 proj GEMM, 4 attention.  slot_mask selects the slots recorded (0 = off); a pool
 * of 16384 event pairs is recycled by mlg_prof_read / mlg_prof_reset, which
 * synchronise the recorded events.  Not for use inside graph capture. */
int mlg_prof_enable(int slot_mask);
int mlg_prof_reset(void);
int mlg_prof_read(int slot, double* total_ms, long* launches);

#ifdef __cplusplus
}
#endif
#endif /* MLGATE_H */
