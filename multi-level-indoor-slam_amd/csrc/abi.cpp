// Public C ABI (include/mlgate.h): ViT-B/14 forward orchestration, kNN gate,
// op-level entry points and HIP-event profiling.
#include <hip/hip_runtime.h>

#include <math.h>

#include <mutex>
#include <vector>

#include "../../include/mlgate.h"
#include <cstddef>

#include "kernels.h"

namespace {

constexpr int PATCH = 14;

inline size_t align_up(size_t v, size_t a = 256) { return (v + a - 1) / a * a; }

struct VitGeom {
    int B, S, grid, P, T, Tpad;
    explicit VitGeom(int b, int s) : B(b), S(s), grid(s / PATCH), P(grid * grid), T(grid * grid + 1) {
        Tpad = (T + 63) / 64 * 64;
    }
};

// Operand buffers are sized for the split-bf16 forward (MLG_VIT_SPLIT): [hi | lo] rows
// for patches / xn / o / h, and q / k / vt as a hi plane followed by a lo plane (lo_elems
// apart); the plain bf16 forward uses the first half of each.
struct VitWorkspace {
    bf16_t *patches, *xn, *q, *k, *vt, *o, *h;
    float *x, *partial;
    int32_t* tasks;  // attention tasks + output offsets, 5 * B int32
    size_t q_bytes, vt_bytes, lo_elems;
};

size_t carve(const VitGeom& g, char* base, VitWorkspace* ws) {
    size_t off = 0;
    auto take = [&](size_t bytes) -> char* {
        char* p = base ? base + off : nullptr;
        off = align_up(off + bytes);
        return p;
    };
    const size_t rows = (size_t)g.B * g.T;
    const size_t heads = (size_t)g.B * 12;
    VitWorkspace w{};
    w.patches = (bf16_t*)take((size_t)g.B * g.P * MLG_VIT_PATCH_K * 2 * 2);
    w.x = (float*)take(rows * 768 * 4);
    w.xn = (bf16_t*)take(rows * 768 * 2 * 2);
    w.lo_elems = heads * g.Tpad * 64;
    w.q_bytes = 2 * w.lo_elems * 2;
    w.q = (bf16_t*)take(w.q_bytes);
    w.k = (bf16_t*)take(2 * w.lo_elems * 2);
    w.vt_bytes = 2 * w.lo_elems * 2;
    w.vt = (bf16_t*)take(w.vt_bytes);
    w.o = (bf16_t*)take(rows * 768 * 2 * 2);
    w.h = (bf16_t*)take(rows * 3072 * 2 * 2);
    w.partial = (float*)take(mlg_gem_partial_bytes(g.B));
    w.tasks = (int32_t*)take((size_t)g.B * 5 * 4);
    if (ws) *ws = w;
    return off;
}

// ------------------------------------------------------------- profiling
struct Prof {
    std::mutex mu;
    unsigned mask = 0;  // slots being recorded
    std::vector<hipEvent_t> pool;
    struct Rec { int slot; hipEvent_t a, b; double work; };
    std::vector<Rec> recs;
    size_t next = 0;
    double total[MLG_PROF_SLOTS] = {0};
    double work[MLG_PROF_SLOTS] = {0};
    long count[MLG_PROF_SLOTS] = {0};
} g_prof;

constexpr size_t PROF_POOL = 32768;

void prof_collect() {
    for (auto& r : g_prof.recs) {
        float ms = 0.f;
        (void)hipEventSynchronize(r.b);
        if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            g_prof.total[r.slot] += ms;
            g_prof.work[r.slot] += r.work;
            g_prof.count[r.slot] += 1;
        }
    }
    g_prof.recs.clear();
    g_prof.next = 0;
}

#define TRY(x)                     \
    do {                           \
        int rc_ = (x);             \
        if (rc_ != MLG_OK) return rc_; \
    } while (0)

}  // namespace

MlgProfScope::MlgProfScope(int slot_, hipStream_t s_, double work_) : slot(slot_), s(s_), work(work_) {
    if (slot < 0 || slot >= MLG_PROF_SLOTS || !(g_prof.mask & (1u << slot))) return;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    if (g_prof.next + 2 > g_prof.pool.size()) return;  // pool exhausted: stop recording
    a = g_prof.pool[g_prof.next++];
    b = g_prof.pool[g_prof.next++];
    (void)hipEventRecord(a, s);
}

MlgProfScope::~MlgProfScope() {
    if (!a) return;
    (void)hipEventRecord(b, s);
    std::lock_guard<std::mutex> lk(g_prof.mu);
    g_prof.recs.push_back({slot, a, b, work});
}

extern "C" {

int mlg_abi_version(void) { return MLG_ABI_VERSION; }

const char* mlg_strerror(int status) {
    switch (status) {
        case MLG_OK: return "ok";
        case MLG_EINVAL: return "invalid argument (shape, alignment or size)";
        case MLG_EHIP: return "HIP launch error";
        case MLG_ENOMEM: return "workspace too small";
        case MLG_ESIZE: return "image size differs from the batch size";
        default: return "unknown mlgate status";
    }
}

size_t mlg_vit_workspace_bytes(int batch, int image_size) {
    if (batch <= 0 || image_size <= 0 || image_size % PATCH) return 0;
    return carve(VitGeom(batch, image_size), nullptr, nullptr);
}

}  // extern "C"

// Preprocess + patch embedding + the 12 blocks; leaves the residual stream in ws->x.
// split: the MLG_VIT_SPLIT forward (weights packed [W_hi | W_lo], 2x the reduction dimension).
static int vit_trunk(const mlg_vit_weights* w, const uint8_t* frames, const VitGeom& g, int H, int W, int C,
                     long frame_stride, int swap_rb, const VitWorkspace& ws, hipStream_t s, int split = 0) {
    const int M = g.B * g.T;
    TRY(mlg_preprocess_patches(frames, g.B, H, W, C, frame_stride, g.S, MLG_VIT_PATCH_K, swap_rb, ws.patches, s,
                               split));
    if (split)
        TRY(mlg_gemm_patch_split(ws.patches, w->patch_w, w->patch_b, w->pos, ws.x, g.B * g.P, g.P, MLG_VIT_PATCH_K,
                                 s));
    else
        TRY(mlg_gemm_patch(ws.patches, w->patch_w, w->patch_b, w->pos, ws.x, g.B * g.P, g.P, MLG_VIT_PATCH_K, s));
    TRY(mlg_cls_rows(ws.x, w->cls, w->pos, g.B, g.T, s));
    // padded key columns of V^T must be finite (masked keys multiply them by p = 0); padded
    // query rows are never stored but are zeroed too, so no lane computes on stale bits
    if (hipMemsetAsync(ws.vt, 0, ws.vt_bytes, s) != hipSuccess) return MLG_EHIP;
    if (hipMemsetAsync(ws.q, 0, ws.q_bytes, s) != hipSuccess) return MLG_EHIP;

    const double mul = split ? 3.0 : 1.0;  // MFMA products per algorithmic product
    for (int l = 0; l < MLG_VIT_DEPTH && split; ++l) {
        const mlg_vit_block& bl = w->blocks[l];
        TRY(mlg_layernorm_split(ws.x, bl.norm1_w, bl.norm1_b, ws.xn, M, s));
        {
            MlgProfScope p(2, s, mul * 2.0 * M * 2304 * 768);
            TRY(mlg_gemm_qkv_split(ws.xn, bl.qkv_w, bl.qkv_b, ws.q, ws.k, ws.vt, M, g.T, g.Tpad, ws.lo_elems, s));
        }
        {
            MlgProfScope p(4, s, mul * 4.0 * g.B * 12 * (double)g.T * g.T * 64);
            TRY(mlg_attention_split(ws.q, ws.k, ws.vt, ws.o, g.B, g.T, g.Tpad, ws.lo_elems, ws.tasks, s));
        }
        {
            MlgProfScope p(3, s, mul * 2.0 * M * 768 * 768);
            TRY(mlg_gemm_residual_split(ws.o, bl.proj_w, bl.proj_b, bl.ls1, ws.x, M, 768, 768, s));
        }
        TRY(mlg_layernorm_split(ws.x, bl.norm2_w, bl.norm2_b, ws.xn, M, s));
        {
            MlgProfScope p(0, s, mul * 2.0 * M * 3072 * 768);
            TRY(mlg_gemm_bias_gelu_split(ws.xn, bl.fc1_w, bl.fc1_b, ws.h, M, 3072, 768, s));
        }
        {
            MlgProfScope p(1, s, mul * 2.0 * M * 768 * 3072);
            TRY(mlg_gemm_residual_split(ws.h, bl.fc2_w, bl.fc2_b, bl.ls2, ws.x, M, 768, 3072, s));
        }
    }
    for (int l = 0; l < MLG_VIT_DEPTH && !split; ++l) {
        const mlg_vit_block& bl = w->blocks[l];
        TRY(mlg_layernorm_bf16(ws.x, bl.norm1_w, bl.norm1_b, ws.xn, M, s));
        {
            MlgProfScope p(2, s, 2.0 * M * 2304 * 768);
            TRY(mlg_gemm_qkv(ws.xn, bl.qkv_w, bl.qkv_b, ws.q, ws.k, ws.vt, M, g.T, g.Tpad, s));
        }
        {
            MlgProfScope p(4, s, 4.0 * g.B * 12 * (double)g.T * g.T * 64);
            TRY(mlg_attention(ws.q, ws.k, ws.vt, ws.o, g.B, g.T, g.Tpad, ws.tasks, s));
        }
        {
            MlgProfScope p(3, s, 2.0 * M * 768 * 768);
            TRY(mlg_gemm_residual(ws.o, bl.proj_w, bl.proj_b, bl.ls1, ws.x, M, 768, 768, s));
        }
        TRY(mlg_layernorm_bf16(ws.x, bl.norm2_w, bl.norm2_b, ws.xn, M, s));
        {
            MlgProfScope p(0, s, 2.0 * M * 3072 * 768);
            TRY(mlg_gemm_bias_gelu_bf16(ws.xn, bl.fc1_w, bl.fc1_b, ws.h, M, 3072, 768, s));
        }
        {
            MlgProfScope p(1, s, 2.0 * M * 768 * 3072);
            TRY(mlg_gemm_residual(ws.h, bl.fc2_w, bl.fc2_b, bl.ls2, ws.x, M, 768, 3072, s));
        }
    }
    return MLG_OK;
}

extern "C" {

int mlg_vit_forward(const mlg_vit_weights* w, const uint8_t* frames, int batch, int H, int W, int C,
                    long frame_stride, int image_size, int flags, void* workspace, size_t workspace_bytes,
                    float* desc_out, float* local_out, void* stream) {
    if (!mlg_head_ok(w, MLG_ABI_VERSION) || !frames || !workspace || !desc_out || batch <= 0 || image_size % PATCH)
        return MLG_EINVAL;
    // the split forward reads 2x-wide weight rows: plain weights with the flag would be read out of bounds
    if (w->packing != ((flags & MLG_VIT_SPLIT) ? MLG_VIT_SPLIT : 0)) return MLG_EINVAL;
    const VitGeom g(batch, image_size);
    VitWorkspace ws;
    if (carve(g, (char*)workspace, &ws) > workspace_bytes) return MLG_ENOMEM;
    hipStream_t s = (hipStream_t)stream;
    const int swap_rb = (flags & MLG_VIT_KEEP_CHANNELS) ? 0 : 1;
    const int mean_pool = (flags & MLG_VIT_POOL_MEAN) ? 1 : 0;
    TRY(vit_trunk(w, frames, g, H, W, C, frame_stride, swap_rb, ws, s, (flags & MLG_VIT_SPLIT) ? 1 : 0));
    TRY(mlg_final_norm_gem(ws.x, w->norm_w, w->norm_b, local_out, ws.partial, desc_out, g.B, g.T, mean_pool, s));
    return MLG_OK;
}

size_t mlg_salad_workspace_bytes(int batch, int image_size) {
    // the head reuses the ViT buffers: hidden [B*T, 1024] bf16 in `h`, scores / cluster
    // features [B*T, 256] f32 in `x` once the final LayerNorm has read it
    return mlg_vit_workspace_bytes(batch, image_size);
}

int mlg_salad_forward(const mlg_vit_weights* w, const mlg_salad_weights* sw, const uint8_t* frames, int batch,
                      int H, int W, int C, long frame_stride, int image_size, void* workspace,
                      size_t workspace_bytes, float* desc_out, void* stream) {
    if (!mlg_head_ok(w, MLG_ABI_VERSION) || !mlg_head_ok(sw, MLG_ABI_VERSION) || !frames || !workspace || !desc_out ||
        batch <= 0 || image_size % PATCH)
        return MLG_EINVAL;
    if (w->packing != 0) return MLG_EINVAL;  // SALAD's trunk runs the plain bf16 forward
    const VitGeom g(batch, image_size);
    VitWorkspace ws;
    if (carve(g, (char*)workspace, &ws) > workspace_bytes) return MLG_ENOMEM;
    hipStream_t s = (hipStream_t)stream;
    const int M = g.B * g.T;
    // SALAD._preprocess keeps the stored channel order (place_recognition.py:395-397)
    TRY(vit_trunk(w, frames, g, H, W, C, frame_stride, /*swap_rb=*/0, ws, s));
    TRY(mlg_layernorm_bf16(ws.x, w->norm_w, w->norm_b, ws.xn, M, s));  // backbone norm_layer, all tokens
    TRY(mlg_gemm_bias_relu_bf16(ws.xn, 768, sw->w1, sw->b1, ws.h, 1024, 1024, M, 1024, 768, s));
    float* y = ws.x;  // [M, 256]
    TRY(mlg_gemm_bias_f32_ld(ws.h, 1024, sw->w2, sw->b2, y, 256, M, 256, 1024, s));
    TRY(mlg_salad_head(ws.xn, y, g.B, g.T, sw->wt1, sw->bt1, sw->wt2, sw->bt2, sw->dust_bin, desc_out, s));
    return MLG_OK;
}

size_t mlg_knn_workspace_bytes(int N, int D, int Q) {
    if (N <= 0 || D <= 0 || Q <= 0) return 0;
    return align_up((size_t)N * D * 4) + align_up((size_t)Q * D * 4) + align_up((size_t)Q * N * 4);
}

// k <= 32 and D % 4 == 0 take the fused scan (no [Q, N] matrix): normalised rows plus
// the per-split partial lists
static bool knn_fused(int D, int k) { return k >= 1 && k <= 32 && D % 4 == 0; }

// fused layouts: gate = Xn | partial lists; query = Xn | Qn | partial lists
size_t mlg_knn_workspace_bytes_k(int N, int D, int Q, int k, int query) {
    if (N <= 0 || D <= 0 || Q <= 0) return 0;
    if (!knn_fused(D, k)) return mlg_knn_workspace_bytes(N, D, Q);
    return align_up((size_t)N * D * 4) + (query ? align_up((size_t)Q * D * 4) : 0) +
           align_up(mlg_knn_fused_ws_bytes(Q, N, k));
}

int mlg_knn_gate(const float* desc, int N, int D, const double* t, const int64_t* floor, const uint8_t* has_floor,
                 double min_gap, float thr, int k, int gating, int q0, int Q, void* workspace,
                 size_t workspace_bytes, int32_t* idx, float* sim, uint8_t* valid, int32_t* count,
                 unsigned long long* totals, void* stream) {
    if (!desc || !t || !workspace || N <= 0 || D <= 0 || Q <= 0 || q0 < 0 || q0 + Q > N) return MLG_EINVAL;
    if (gating && (!floor || !has_floor)) return MLG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    float* Xn = (float*)workspace;
    float* S = (float*)((char*)workspace + align_up((size_t)N * D * 4) + align_up((size_t)Q * D * 4));
    if (knn_fused(D, k)) {
        if (mlg_knn_workspace_bytes_k(N, D, Q, k, 0) > workspace_bytes) return MLG_ENOMEM;
        TRY(mlg_row_normalize_wave(desc, Xn, N, D, nullptr, s));
        void* part = (char*)workspace + align_up((size_t)N * D * 4);
        return mlg_knn_fused(Xn + (size_t)q0 * D, Q, Xn, N, D, t + q0, t, gating ? floor + q0 : nullptr,
                             gating ? has_floor + q0 : nullptr, gating ? floor : nullptr, gating ? has_floor : nullptr,
                             min_gap, thr, k, gating, part, idx, sim, valid, count, totals, s);
    }
    if (mlg_knn_workspace_bytes(N, D, Q) > workspace_bytes) return MLG_ENOMEM;
    TRY(mlg_row_normalize(desc, Xn, N, D, nullptr, s));
    TRY(mlg_similarity_f32(Xn + (size_t)q0 * D, Q, Xn, N, D, S, N, s));
    TRY(mlg_topk_gate(S, N, N, Q, t + q0, t, gating ? floor + q0 : nullptr, gating ? has_floor + q0 : nullptr,
                      gating ? floor : nullptr, gating ? has_floor : nullptr, min_gap, thr, k, gating, idx, sim,
                      valid, count, totals, s));
    return MLG_OK;
}

int mlg_knn_query(const float* db, int N, int D, const float* qdesc, int Q, const double* t_db,
                  const double* t_query, double min_gap, int k, void* workspace, size_t workspace_bytes,
                  int32_t* idx, float* sim, int32_t* count, void* stream) {
    if (!db || !qdesc || !t_db || !t_query || !workspace || N <= 0 || D <= 0 || Q <= 0) return MLG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    float* Xn = (float*)workspace;
    float* Qn = (float*)((char*)workspace + align_up((size_t)N * D * 4));
    float* S = (float*)((char*)Qn + align_up((size_t)Q * D * 4));
    if (knn_fused(D, k)) {
        if (mlg_knn_workspace_bytes_k(N, D, Q, k, 1) > workspace_bytes) return MLG_ENOMEM;
        TRY(mlg_row_normalize_wave(db, Xn, N, D, nullptr, s));
        TRY(mlg_row_normalize_wave(qdesc, Qn, Q, D, nullptr, s));
        return mlg_knn_fused(Qn, Q, Xn, N, D, t_query, t_db, nullptr, nullptr, nullptr, nullptr, min_gap, -INFINITY,
                             k, 0, S, idx, sim, nullptr, count, nullptr, s);
    }
    if (mlg_knn_workspace_bytes(N, D, Q) > workspace_bytes) return MLG_ENOMEM;
    TRY(mlg_row_normalize(db, Xn, N, D, nullptr, s));
    TRY(mlg_row_normalize(qdesc, Qn, Q, D, nullptr, s));
    TRY(mlg_similarity_f32(Qn, Q, Xn, N, D, S, N, s));
    TRY(mlg_topk_gate(S, N, N, Q, t_query, t_db, nullptr, nullptr, nullptr, nullptr, min_gap, -INFINITY, k, 0, idx,
                      sim, nullptr, count, nullptr, s));
    return MLG_OK;
}

int mlg_row_normalize_f32(const float* X, float* Xn, int N, int D, float* norms_or_null, void* stream) {
    return mlg_row_normalize(X, Xn, N, D, norms_or_null, (hipStream_t)stream);
}

int mlg_similarity(const float* A, int Q, const float* B, int N, int D, float* S, void* stream) {
    return mlg_similarity_f32(A, Q, B, N, D, S, N, (hipStream_t)stream);
}

size_t mlg_plane_ransac_workspace_bytes(int S, int iterations) { return mlg_plane_ws_bytes(S, iterations); }

int mlg_plane_ransac(const float* pts, const int32_t* offsets, int S, int iterations, uint64_t seed, double threshold,
                     void* workspace, size_t workspace_bytes, double* plane, double* ratio, int32_t* inliers,
                     void* stream) {
    if (!pts || !offsets || !workspace || !plane || !ratio || !inliers) return MLG_EINVAL;
    return mlg_plane_ransac_run(pts, offsets, S, iterations, seed, threshold, workspace, workspace_bytes, plane,
                                ratio, inliers, (hipStream_t)stream);
}

size_t mlg_proximity_workspace_bytes(int N, int nrows) { return mlg_proximity_ws_bytes(N, nrows); }

int mlg_proximity_count(const double* pos, const int64_t* floor, int N, int row0, int nrows, double radius,
                        int min_gap, int strict, void* workspace, size_t workspace_bytes, long long* totals,
                        void* stream) {
    if ((!pos && N > 0) || !workspace || !totals) return MLG_EINVAL;
    return mlg_proximity_count_run(pos, floor, N, row0, nrows, radius, min_gap, strict, workspace, workspace_bytes,
                                   totals, (hipStream_t)stream);
}

int mlg_proximity_emit(const double* pos, const int64_t* floor, int N, int row0, int nrows, double radius,
                       int min_gap, int strict, const void* workspace, size_t workspace_bytes, int32_t* pairs,
                       double* dist, uint8_t* valid, void* stream) {
    if ((!pos && N > 0) || !workspace || !pairs || !dist || !valid) return MLG_EINVAL;
    return mlg_proximity_emit_run(pos, floor, N, row0, nrows, radius, min_gap, strict, workspace, workspace_bytes,
                                  pairs, dist, valid, (hipStream_t)stream);
}

// the internal tables are the public structs past their 8-byte head
static_assert(offsetof(mlg_rn_weights, stem_w) == 8 &&
                  sizeof(mlg_rn_weights) - offsetof(mlg_rn_weights, stem_w) == sizeof(mlg_rn_weights_i),
              "ResNet weight tables must match");

size_t mlg_resnet50_workspace_bytes(int B, int H, int W) { return mlg_resnet50_ws_bytes(B, H, W); }

int mlg_resnet50_forward(const mlg_rn_weights* w, const uint8_t* frames, int B, int H, int W, int C,
                         long frame_stride, int descriptor_dim, void* workspace, size_t workspace_bytes,
                         float* desc, void* stream) {
    if (!mlg_head_ok(w, MLG_ABI_VERSION) || !frames || !workspace || !desc || !w->stem_w || !w->stem_b)
        return MLG_EINVAL;
    for (int i = 0; i < 16; ++i) {
        const mlg_rn_block& b = w->blocks[i];
        if (!b.w1 || !b.b1 || !b.w2 || !b.b2 || !b.w3 || !b.b3) return MLG_EINVAL;
        const bool first = i == 0 || i == 3 || i == 7 || i == 13;
        if (first != (b.wd != nullptr) || (b.wd && !b.bd)) return MLG_EINVAL;
    }
    if (frame_stride < (long)H * W * C) return MLG_EINVAL;
    return mlg_resnet50_run(*reinterpret_cast<const mlg_rn_weights_i*>(&w->stem_w), frames, B, H, W, C, frame_stride,
                            descriptor_dim, workspace, workspace_bytes, desc, nullptr, (hipStream_t)stream);
}

int mlg_op_pillow_resize_224(const uint8_t* frames, int B, int H, int W, int C, long frame_stride, void* workspace,
                             size_t workspace_bytes, uint8_t* out, void* stream) {
    if (!frames || !workspace || !out || frame_stride < (long)H * W * C) return MLG_EINVAL;
    mlg_rn_weights_i none{};
    return mlg_resnet50_run(none, frames, B, H, W, C, frame_stride, 1, workspace, workspace_bytes, nullptr, out,
                            (hipStream_t)stream);
}

size_t mlg_superpoint_workspace_bytes(int B, int H, int W) { return mlg_superpoint_ws_bytes(B, H, W); }

int mlg_superpoint(const mlg_sp_weights* w, const uint8_t* frames, int B, int H, int W, int C, long frame_stride,
                   float detection_threshold, int max_keypoints, int nms_radius, int remove_borders, void* workspace,
                   size_t workspace_bytes, float* keypoints, float* scores, float* descriptors,
                   uint16_t* descriptors_bf16, int32_t* counts, void* stream) {
    if (!mlg_head_ok(w, MLG_ABI_VERSION) || !frames || !workspace || !keypoints || !scores || !descriptors || !counts)
        return MLG_EINVAL;
    if (!w->conv1a_w || !w->conv1a_b) return MLG_EINVAL;
    mlg_sp_weights_i wi;
    wi.conv1a_w = w->conv1a_w;
    wi.conv1a_b = w->conv1a_b;
    for (int i = 0; i < 11; ++i) {
        if (!w->w[i] || !w->b[i]) return MLG_EINVAL;
        if ((reinterpret_cast<uintptr_t>(w->w[i]) & 15) || (reinterpret_cast<uintptr_t>(w->b[i]) & 15))
            return MLG_EINVAL;
        wi.w[i] = (const bf16_t*)w->w[i];
        wi.b[i] = w->b[i];
    }
    if (frame_stride < (long)H * W * C) return MLG_EINVAL;
    return mlg_superpoint_run(wi, frames, B, H, W, C, frame_stride, detection_threshold, max_keypoints, nms_radius,
                              remove_borders, workspace, workspace_bytes, keypoints, scores, descriptors,
                              descriptors_bf16, counts, (hipStream_t)stream);
}

static_assert(offsetof(mlg_lg_weights, Wr) == 8 &&
                  sizeof(mlg_lg_weights) - offsetof(mlg_lg_weights, Wr) == sizeof(mlg_lg_weights_i),
              "LightGlue weight tables must match");
static_assert(sizeof(mlg_lg_block) == sizeof(mlg_lg_block_i), "LightGlue block tables must match");

size_t mlg_lightglue_workspace_bytes(int P, int kmax) { return mlg_lightglue_ws_bytes(P, kmax); }

int mlg_lightglue(const mlg_lg_weights* w, const float* keypoints, const float* descriptors, const int32_t* counts,
                  int F, int kmax, const int32_t* pair_a, const int32_t* pair_b, int P, float depth_confidence,
                  float width_confidence, float filter_threshold, int pruning_min_kpts, void* workspace,
                  size_t workspace_bytes, int32_t* matches, float* scores, int32_t* num_matches, int32_t* stop_layer,
                  void* stream) {
    if (!mlg_head_ok(w, MLG_ABI_VERSION) || !keypoints || !descriptors || !counts || !pair_a || !pair_b || !workspace ||
        !matches || !scores || !num_matches || F <= 0 || P <= 0)
        return MLG_EINVAL;
    for (int p = 0; p < P; ++p)
        if (pair_a[p] < 0 || pair_a[p] >= F || pair_b[p] < 0 || pair_b[p] >= F) return MLG_EINVAL;
    const mlg_lg_weights_i& wi = *reinterpret_cast<const mlg_lg_weights_i*>(&w->Wr);
    return mlg_lightglue_run(wi, keypoints, descriptors, counts, kmax, pair_a, pair_b, P, depth_confidence,
                             width_confidence, filter_threshold, pruning_min_kpts, workspace, workspace_bytes,
                             matches, scores, num_matches, stop_layer, (hipStream_t)stream);
}

static_assert(offsetof(mlg_sg_weights, kenc_w) == 8 &&
                  sizeof(mlg_sg_weights) - offsetof(mlg_sg_weights, kenc_w) == sizeof(mlg_sg_weights_i),
              "SuperGlue weight tables must match");

size_t mlg_superglue_workspace_bytes(int P, int kmax) { return mlg_superglue_ws_bytes(P, kmax); }

int mlg_superglue(const mlg_sg_weights* w, const float* keypoints, const float* scores, const float* descriptors,
                  const int32_t* counts, int F, int kmax, int W, int H, const int32_t* pair_a, const int32_t* pair_b,
                  int P, int sinkhorn_iterations, float match_threshold, void* workspace, size_t workspace_bytes,
                  int32_t* matches, float* match_scores, int32_t* num_matches, void* stream) {
    if (!mlg_head_ok(w, MLG_ABI_VERSION) || !keypoints || !scores || !descriptors || !counts || !pair_a || !pair_b ||
        !workspace || !matches || !match_scores || !num_matches || F <= 0 || P <= 0 || W <= 0 || H <= 0)
        return MLG_EINVAL;
    for (int p = 0; p < P; ++p)
        if (pair_a[p] < 0 || pair_a[p] >= F || pair_b[p] < 0 || pair_b[p] >= F) return MLG_EINVAL;
    const mlg_sg_weights_i& wi = *reinterpret_cast<const mlg_sg_weights_i*>(&w->kenc_w);
    return mlg_superglue_run(wi, keypoints, scores, descriptors, counts, kmax, W, H, pair_a, pair_b, P,
                             sinkhorn_iterations, match_threshold, workspace, workspace_bytes, matches, match_scores,
                             num_matches, (hipStream_t)stream);
}

size_t mlg_ransac_workspace_bytes(int P, long S_total, int hypotheses) {
    return mlg_ransac_ws_bytes(P, S_total, hypotheses);
}

int mlg_ransac_epipolar(const float* kp1, const float* kp2, const int32_t* offsets, int P, long S_total,
                        const double* K, int k_stride, double threshold, int hypotheses, uint64_t seed,
                        void* workspace, size_t workspace_bytes, double* model, uint8_t* mask, int32_t* inliers,
                        double* pose, int32_t* status, void* stream) {
    if (!offsets || !workspace || !model || !inliers || !status || (S_total > 0 && (!kp1 || !kp2 || !mask)))
        return MLG_EINVAL;
    if (K && k_stride != 0 && k_stride != 9) return MLG_EINVAL;
    return mlg_ransac_run(kp1, kp2, offsets, P, S_total, K, k_stride, threshold, hypotheses, seed, workspace,
                          workspace_bytes, model, mask, inliers, pose, status, (hipStream_t)stream);
}

int mlg_recover_pose(const float* kp1, const float* kp2, const int32_t* offsets, int P, const double* K,
                     int k_stride, const double* E, const uint8_t* mask, double* pose, void* stream) {
    if (!kp1 || !kp2 || !offsets || !K || !E || !mask || !pose) return MLG_EINVAL;
    if (k_stride != 0 && k_stride != 9) return MLG_EINVAL;
    return mlg_recover_pose_run(kp1, kp2, offsets, P, K, k_stride, E, mask, pose, (hipStream_t)stream);
}

size_t mlg_xcorr_workspace_bytes(int n1, int n2, int D) {
    if (n1 <= 0 || n2 <= 0 || D <= 0) return 0;
    return align_up((size_t)n1 * D * 4) + align_up((size_t)n2 * D * 4) + align_up((size_t)n1 * n2 * 4);
}

int mlg_xcorr_score(const float* q, int n1, const float* m, int n2, int D, void* workspace, size_t workspace_bytes,
                    float* score, void* stream) {
    if (!q || !m || !workspace || !score || n1 <= 0 || n2 <= 0 || D <= 0) return MLG_EINVAL;
    if (mlg_xcorr_workspace_bytes(n1, n2, D) > workspace_bytes) return MLG_ENOMEM;
    hipStream_t s = (hipStream_t)stream;
    float* qn = (float*)workspace;
    float* mn = (float*)((char*)workspace + align_up((size_t)n1 * D * 4));
    float* C = (float*)((char*)mn + align_up((size_t)n2 * D * 4));
    TRY(mlg_row_normalize(q, qn, n1, D, nullptr, s));
    TRY(mlg_row_normalize(m, mn, n2, D, nullptr, s));
    TRY(mlg_similarity_f32(qn, n1, mn, n2, D, C, n2, s));
    TRY(mlg_xcorr_reduce(C, n1, n2, score, s));
    return MLG_OK;
}

size_t mlg_xcorr_batch_workspace_bytes(int F, int L, int D, int P) { return mlg_xcorr_batch_ws_bytes(F, L, D, P); }

int mlg_xcorr_batch(const float* feats, int F, int L, int D, const int32_t* query, const int32_t* cand, int P,
                    void* workspace, size_t workspace_bytes, float* scores, void* stream) {
    return mlg_xcorr_batch_run(feats, F, L, D, query, cand, P, workspace, workspace_bytes, scores,
                               (hipStream_t)stream);
}

int mlg_op_gemm_f32out(const uint16_t* A, const uint16_t* W, float* C, int M, int N, int K, void* stream) {
    return mlg_gemm_f32out(A, W, C, M, N, K, (hipStream_t)stream);
}
int mlg_op_gemm_f32out_variant(int variant, const uint16_t* A, const uint16_t* W, float* C, int M, int N, int K,
                               void* stream) {
    return mlg_gemm_f32out_variant(variant, A, W, C, M, N, K, (hipStream_t)stream);
}
int mlg_set_gemm_variant(int variant) { return mlg_gemm_set_variant(variant); }
int mlg_op_gemm_bias_gelu(const uint16_t* A, const uint16_t* W, const float* bias, uint16_t* C, int M, int N,
                          int K, void* stream) {
    return mlg_gemm_bias_gelu_bf16(A, W, bias, C, M, N, K, (hipStream_t)stream);
}
int mlg_op_gemm_residual(const uint16_t* A, const uint16_t* W, const float* bias, const float* gamma, float* X,
                         int M, int N, int K, void* stream) {
    return mlg_gemm_residual(A, W, bias, gamma, X, M, N, K, (hipStream_t)stream);
}
int mlg_op_layernorm_bf16(const float* X, const float* g, const float* b, uint16_t* Y, int M, void* stream) {
    return mlg_layernorm_bf16(X, g, b, Y, M, (hipStream_t)stream);
}
int mlg_op_attention(const uint16_t* Q, const uint16_t* K, const uint16_t* Vt, uint16_t* O, int B, int T, int Tpad,
                     int32_t* task_ws, void* stream) {
    return mlg_attention(Q, K, Vt, O, B, T, Tpad, task_ws, (hipStream_t)stream);
}
int mlg_op_attention_varlen(const uint16_t* Q, const uint16_t* K, const uint16_t* Vt, uint16_t* O, int ldo, int Npad,
                            int heads, const int32_t* tasks, const int32_t* out_off, int ntasks, int max_q,
                            void* stream) {
    return mlg_attention_varlen(Q, K, Vt, O, ldo, Npad, heads, reinterpret_cast<const int4*>(tasks), out_off, ntasks,
                                max_q, (hipStream_t)stream);
}
int mlg_op_lg_ffn(const uint16_t* ctx, float* X, uint16_t* xcopy, int ldc, int M, const uint16_t* Wout,
                  const float* bout, const uint16_t* Wf1, const float* bf1, const float* ln_g, const float* ln_b,
                  const uint16_t* Wf2, const float* bf2, void* stream) {
    mlg_lg_block_i w{};
    w.Wout = Wout; w.bout = bout; w.Wf1 = Wf1; w.bf1 = bf1; w.ln_g = ln_g; w.ln_b = ln_b; w.Wf2 = Wf2; w.bf2 = bf2;
    return mlg_lg_ffn(ctx, X, xcopy, ldc, M, w, (hipStream_t)stream);
}
int mlg_op_lg_proj(int self_block, const uint16_t* xcopy, int ldx, const uint16_t* W, const float* bias,
                   const float* ecos, const float* esin, const uint8_t* live, uint16_t* Q, uint16_t* K, uint16_t* Vt,
                   int Npad, void* stream) {
    (void)esin;  // the factors come interleaved in `ecos` (lg_fac4 layout, include/mlgate.h)
    return mlg_lg_proj(self_block != 0, xcopy, ldx, W, bias, ecos, live, Q, K, Vt, Npad, (hipStream_t)stream);
}
int mlg_op_conv2d_nhwc(const uint16_t* in, const uint16_t* zero16, int B, int H, int W, int C, int k, int s,
                       const uint16_t* Wt, const float* bias, float* out, int N, void* stream) {
    return mlg_conv_implicit(in, zero16, B, H, W, C, k, s, Wt, bias, nullptr, 0, out, N, nullptr, 0, 0, N, N,
                             (hipStream_t)stream);
}
int mlg_op_preprocess_patches(const uint8_t* frames, int B, int H, int W, int C, long frame_stride, int S,
                              uint16_t* patches, void* stream) {
    return mlg_preprocess_patches(frames, B, H, W, C, frame_stride, S, MLG_VIT_PATCH_K, 1, patches,
                                  (hipStream_t)stream);
}

int mlg_prof_enable(int slot_mask) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    if (slot_mask && g_prof.pool.empty()) {
        g_prof.pool.resize(PROF_POOL);
        for (auto& e : g_prof.pool)
            if (hipEventCreate(&e) != hipSuccess) return MLG_EHIP;
    }
    g_prof.mask = (unsigned)slot_mask & ((1u << MLG_PROF_SLOTS) - 1);
    return MLG_OK;
}

int mlg_prof_reset(void) {
    std::lock_guard<std::mutex> lk(g_prof.mu);
    prof_collect();
    for (int i = 0; i < MLG_PROF_SLOTS; ++i) {
        g_prof.total[i] = 0;
        g_prof.work[i] = 0;
        g_prof.count[i] = 0;
    }
    return MLG_OK;
}

int mlg_prof_read(int slot, double* total_ms, long* launches) {
    if (slot < 0 || slot >= MLG_PROF_SLOTS || !total_ms || !launches) return MLG_EINVAL;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    prof_collect();
    *total_ms = g_prof.total[slot];
    *launches = g_prof.count[slot];
    return MLG_OK;
}

int mlg_prof_read_work(int slot, double* flops) {
    if (slot < 0 || slot >= MLG_PROF_SLOTS || !flops) return MLG_EINVAL;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    prof_collect();
    *flops = g_prof.work[slot];
    return MLG_OK;
}

}  // extern "C"
