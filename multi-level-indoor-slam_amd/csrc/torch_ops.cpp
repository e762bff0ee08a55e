#include <cstdlib>
// PyTorch-ROCm custom operators over the mlgate C ABI (include/mlgate.h).
//
// TORCH_LIBRARY(mlgate, m) declares one operator per ABI entry point the Python
// drop-in uses (mlgate/*.py call torch.ops.mlgate.*); TORCH_LIBRARY_IMPL(mlgate, CUDA, m)
// binds them for HIP tensors (PyTorch-ROCm names its HIP dispatch key CUDA).  Each
// operator checks devices / dtypes / shapes, allocates its outputs and workspace from
// the caching allocator and launches on the current HIP stream of the tensors' device,
// so the ops compose with torch streams, events and hipGraph capture (the ABI itself
// never allocates or synchronises; LightGlue and the proximity emit read one small
// device result back by design -- see the header).  Weights arrive as flat tensor
// lists in the order of the ABI's weight structs (mlgate/*.py build them once).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cstring>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/mlgate.h"

namespace {

using at::Tensor;

void check_rc(int rc, const char* what) { TORCH_CHECK(rc == MLG_OK, what, " failed: ", mlg_strerror(rc)); }

void* stream_of(const Tensor& t) { return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void want(const Tensor& t, at::ScalarType ty, const char* name, bool device = true) {
    TORCH_CHECK(t.scalar_type() == ty, name, ": expected ", ty, ", got ", t.scalar_type());
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    if (device) {
        TORCH_CHECK(t.is_cuda(), name, " must be on the HIP device");
    } else {
        TORCH_CHECK(t.device().is_cpu(), name, " must be a host tensor");
    }
}

template <typename T>
const T* cp(const Tensor& t) {
    return t.defined() && t.numel() > 0 ? reinterpret_cast<const T*>(t.data_ptr()) : nullptr;
}
template <typename T>
T* mp(const Tensor& t) {
    return t.defined() && t.numel() > 0 ? reinterpret_cast<T*>(t.data_ptr()) : nullptr;
}

Tensor workspace(size_t bytes, const Tensor& like) {
    Tensor t = at::empty({(int64_t)std::max<size_t>(bytes, 1)}, like.options().dtype(at::kByte));
    // diagnostic (MLG_WS_POISON=1): every workspace starts as all-ones bytes (NaN in f32 /
    // bf16), so a kernel that reads workspace it never wrote shows up as changed results
    static const bool poison = [] {
        const char* v = getenv("MLG_WS_POISON");
        return v && atoi(v) != 0;
    }();
    if (poison) t.fill_(255);
    return t;
}

// ------------------------------------------------------------------ ViT-B/14
constexpr int kVitBlockTensors = 14;
constexpr int kVitTensors = 4 + MLG_VIT_DEPTH * kVitBlockTensors + 2;

// split: weights packed for MLG_VIT_SPLIT ([W_hi | W_lo], 2x the reduction dim)
mlg_vit_weights vit_weights(const std::vector<Tensor>& w, bool split = false) {
    TORCH_CHECK((int)w.size() == kVitTensors, "vit weights: expected ", kVitTensors, " tensors, got ", w.size());
    const int64_t m = split ? 2 : 1;
    auto want_n = [&](const Tensor& t, int64_t n, const char* what) {
        TORCH_CHECK(t.numel() == n * m && t.scalar_type() == at::kBFloat16, "vit weights: ", what, " must be bf16 with ",
                    n * m, " elements", split ? " (split packing)" : "");
    };
    want_n(w[0], 768LL * MLG_VIT_PATCH_K, "patch_w");
    for (int i = 0; i < MLG_VIT_DEPTH; ++i) {
        const Tensor* b = &w[4 + i * kVitBlockTensors];
        want_n(b[2], 2304LL * 768, "qkv_w");
        want_n(b[4], 768LL * 768, "proj_w");
        want_n(b[9], 3072LL * 768, "fc1_w");
        want_n(b[11], 768LL * 3072, "fc2_w");
    }
    mlg_vit_weights s = MLG_STRUCT_INIT(mlg_vit_weights);
    s.patch_w = cp<uint16_t>(w[0]);
    s.patch_b = cp<float>(w[1]);
    s.cls = cp<float>(w[2]);
    s.pos = cp<float>(w[3]);
    for (int i = 0; i < MLG_VIT_DEPTH; ++i) {
        const Tensor* b = &w[4 + i * kVitBlockTensors];
        mlg_vit_block& o = s.blocks[i];
        o.norm1_w = cp<float>(b[0]); o.norm1_b = cp<float>(b[1]);
        o.qkv_w = cp<uint16_t>(b[2]); o.qkv_b = cp<float>(b[3]);
        o.proj_w = cp<uint16_t>(b[4]); o.proj_b = cp<float>(b[5]); o.ls1 = cp<float>(b[6]);
        o.norm2_w = cp<float>(b[7]); o.norm2_b = cp<float>(b[8]);
        o.fc1_w = cp<uint16_t>(b[9]); o.fc1_b = cp<float>(b[10]);
        o.fc2_w = cp<uint16_t>(b[11]); o.fc2_b = cp<float>(b[12]); o.ls2 = cp<float>(b[13]);
    }
    s.norm_w = cp<float>(w[kVitTensors - 2]);
    s.norm_b = cp<float>(w[kVitTensors - 1]);
    s.packing = split ? MLG_VIT_SPLIT : 0;
    return s;
}

// frames uint8 [B, H, W, C]; writes desc f32 [B, 768] and local f32 [B, n_local, 768]
void vit_forward_into(const Tensor& frames, at::TensorList w, int64_t image_size, int64_t flags, int64_t max_batch,
                      const Tensor& desc, const c10::optional<Tensor>& local) {
    want(frames, at::kByte, "frames");
    TORCH_CHECK(frames.dim() == 4, "frames must be [B, H, W, C]");
    want(desc, at::kFloat, "desc");
    const int64_t B = frames.size(0), H = frames.size(1), W = frames.size(2), C = frames.size(3);
    TORCH_CHECK(desc.dim() == 2 && desc.size(0) == B && desc.size(1) == MLG_VIT_EMBED, "desc must be [B, 768]");
    const int64_t grid = image_size / 14, n_local = grid * grid - 1;
    if (local.has_value() && local->defined()) {
        want(*local, at::kFloat, "local");
        TORCH_CHECK(local->dim() == 3 && local->size(0) == B && local->size(1) == n_local &&
                        local->size(2) == MLG_VIT_EMBED, "local must be [B, (S/14)^2 - 1, 768]");
    }
    TORCH_CHECK(max_batch > 0, "max_batch must be positive");
    std::vector<Tensor> wv(w.begin(), w.end());
    const mlg_vit_weights s = vit_weights(wv, (flags & MLG_VIT_SPLIT) != 0);
    c10::DeviceGuard g(frames.device());
    const int64_t nb_max = std::min(B, max_batch);
    Tensor ws = workspace(mlg_vit_workspace_bytes((int)nb_max, (int)image_size), frames);
    const long stride = (long)(H * W * C);
    for (int64_t b0 = 0; b0 < B; b0 += max_batch) {
        const int nb = (int)std::min(max_batch, B - b0);
        float* lo = (local.has_value() && local->defined()) ? mp<float>(*local) + b0 * n_local * MLG_VIT_EMBED
                                                           : nullptr;
        check_rc(mlg_vit_forward(&s, cp<uint8_t>(frames) + b0 * stride, nb, (int)H, (int)W, (int)C, stride,
                                 (int)image_size, (int)flags, ws.data_ptr(), (size_t)ws.numel(),
                                 mp<float>(desc) + b0 * MLG_VIT_EMBED, lo, stream_of(frames)),
                 "mlg_vit_forward");
    }
}

// SALAD: frames uint8 [B, H, W, C] -> desc f32 [B, 8448]; salad = [w1, b1, w2, b2, wt1, bt1, wt2, bt2]
Tensor salad_forward(const Tensor& frames, at::TensorList w, at::TensorList salad, double dust_bin,
                     int64_t image_size, int64_t max_batch) {
    want(frames, at::kByte, "frames");
    TORCH_CHECK(frames.dim() == 4, "frames must be [B, H, W, C]");
    TORCH_CHECK(salad.size() == 8, "salad weights: expected 8 tensors");
    TORCH_CHECK(max_batch > 0, "max_batch must be positive");
    const int64_t B = frames.size(0), H = frames.size(1), W = frames.size(2), C = frames.size(3);
    std::vector<Tensor> wv(w.begin(), w.end());
    const mlg_vit_weights s = vit_weights(wv);
    const at::ScalarType kinds[8] = {at::kBFloat16, at::kFloat, at::kBFloat16, at::kFloat,
                                     at::kFloat,    at::kFloat, at::kFloat,    at::kFloat};
    const int64_t numel[8] = {1024 * 768, 1024, 256 * 1024, 256, 512 * 768, 512, 256 * 512, 256};
    for (int i = 0; i < 8; ++i) {
        want(salad[i], kinds[i], "salad weight");
        TORCH_CHECK(salad[i].numel() == numel[i], "salad weight ", i, ": expected ", numel[i], " elements");
    }
    mlg_salad_weights sw = MLG_STRUCT_INIT(mlg_salad_weights);
    sw.w1 = cp<uint16_t>(salad[0]); sw.b1 = cp<float>(salad[1]);
    sw.w2 = cp<uint16_t>(salad[2]); sw.b2 = cp<float>(salad[3]);
    sw.wt1 = cp<float>(salad[4]); sw.bt1 = cp<float>(salad[5]);
    sw.wt2 = cp<float>(salad[6]); sw.bt2 = cp<float>(salad[7]);
    sw.dust_bin = (float)dust_bin;
    c10::DeviceGuard g(frames.device());
    Tensor desc = at::empty({B, MLG_SALAD_DIM}, frames.options().dtype(at::kFloat));
    const int64_t nb_max = std::min(B, max_batch);
    Tensor ws = workspace(mlg_salad_workspace_bytes((int)nb_max, (int)image_size), frames);
    const long stride = (long)(H * W * C);
    for (int64_t b0 = 0; b0 < B; b0 += max_batch) {
        const int nb = (int)std::min(max_batch, B - b0);
        check_rc(mlg_salad_forward(&s, &sw, cp<uint8_t>(frames) + b0 * stride, nb, (int)H, (int)W, (int)C, stride,
                                   (int)image_size, ws.data_ptr(), (size_t)ws.numel(),
                                   mp<float>(desc) + b0 * MLG_SALAD_DIM, stream_of(frames)),
                 "mlg_salad_forward");
    }
    return desc;
}

// --------------------------------------------------------------- retrieval
std::tuple<Tensor, Tensor, Tensor, Tensor> knn_gate(const Tensor& desc, const Tensor& t, const Tensor& floor,
                                                    const Tensor& has_floor, double min_gap, double thr, int64_t k,
                                                    bool gating, int64_t q0, int64_t Q,
                                                    const c10::optional<Tensor>& totals) {
    want(desc, at::kFloat, "desc");
    want(t, at::kDouble, "t");
    want(floor, at::kLong, "floor");
    want(has_floor, at::kByte, "has_floor");
    TORCH_CHECK(desc.dim() == 2, "desc must be [N, D]");
    const int64_t N = desc.size(0), D = desc.size(1);
    TORCH_CHECK(t.numel() == N && floor.numel() == N && has_floor.numel() == N, "t / floor / has_floor must be [N]");
    TORCH_CHECK(k >= 1, "k must be >= 1");
    TORCH_CHECK(q0 >= 0 && Q >= 0 && q0 + Q <= N, "query rows out of range");
    if (totals.has_value() && totals->defined()) {
        want(*totals, at::kLong, "totals");
        TORCH_CHECK(totals->numel() == 2, "totals must be int64 [2]");
    }
    c10::DeviceGuard g(desc.device());
    auto o = desc.options();
    Tensor idx = at::empty({Q, k}, o.dtype(at::kInt)), sim = at::empty({Q, k}, o.dtype(at::kFloat));
    Tensor valid = at::empty({Q, k}, o.dtype(at::kByte)), count = at::empty({Q}, o.dtype(at::kInt));
    Tensor ws = workspace(mlg_knn_workspace_bytes_k((int)N, (int)D, (int)Q, (int)k, 0), desc);
    check_rc(mlg_knn_gate(cp<float>(desc), (int)N, (int)D, cp<double>(t), cp<int64_t>(floor), cp<uint8_t>(has_floor),
                          min_gap, (float)thr, (int)k, gating ? 1 : 0, (int)q0, (int)Q, ws.data_ptr(),
                          (size_t)ws.numel(), mp<int32_t>(idx), mp<float>(sim), mp<uint8_t>(valid), mp<int32_t>(count),
                          (totals.has_value() && totals->defined()) ? mp<unsigned long long>(*totals) : nullptr,
                          stream_of(desc)),
             "mlg_knn_gate");
    return {idx, sim, valid, count};
}

std::tuple<Tensor, Tensor, Tensor> knn_query(const Tensor& db, const Tensor& q, const Tensor& t_db,
                                             const Tensor& t_q, double min_gap, int64_t k) {
    want(db, at::kFloat, "db");
    want(q, at::kFloat, "q");
    want(t_db, at::kDouble, "t_db");
    want(t_q, at::kDouble, "t_q");
    const int64_t N = db.size(0), D = db.size(1), Q = q.size(0);
    TORCH_CHECK(q.dim() == 2 && q.size(1) == D && t_db.numel() == N && t_q.numel() == Q, "knn_query shapes");
    TORCH_CHECK(k >= 1, "k must be >= 1");
    c10::DeviceGuard g(db.device());
    auto o = db.options();
    Tensor idx = at::empty({Q, k}, o.dtype(at::kInt)), sim = at::empty({Q, k}, o.dtype(at::kFloat));
    Tensor count = at::empty({Q}, o.dtype(at::kInt));
    Tensor ws = workspace(mlg_knn_workspace_bytes_k((int)N, (int)D, (int)Q, (int)k, 1), db);
    check_rc(mlg_knn_query(cp<float>(db), (int)N, (int)D, cp<float>(q), (int)Q, cp<double>(t_db), cp<double>(t_q),
                           min_gap, (int)k, ws.data_ptr(), (size_t)ws.numel(), mp<int32_t>(idx), mp<float>(sim),
                           mp<int32_t>(count), stream_of(db)),
             "mlg_knn_query");
    return {idx, sim, count};
}

Tensor row_normalize(const Tensor& X) {
    want(X, at::kFloat, "X");
    TORCH_CHECK(X.dim() == 2, "X must be [N, D]");
    c10::DeviceGuard g(X.device());
    Tensor Y = at::empty_like(X);
    check_rc(mlg_row_normalize_f32(cp<float>(X), mp<float>(Y), (int)X.size(0), (int)X.size(1), nullptr, stream_of(X)),
             "mlg_row_normalize_f32");
    return Y;
}

// S = A . B^T of row-normalised A [Q, D], B [N, D] (float32)
Tensor similarity(const Tensor& A, const Tensor& B) {
    want(A, at::kFloat, "A");
    want(B, at::kFloat, "B");
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "similarity shapes");
    c10::DeviceGuard g(A.device());
    Tensor S = at::empty({A.size(0), B.size(0)}, A.options());
    check_rc(mlg_similarity(cp<float>(A), (int)A.size(0), cp<float>(B), (int)B.size(0), (int)A.size(1), mp<float>(S),
                            stream_of(A)),
             "mlg_similarity");
    return S;
}

Tensor xcorr_score(const Tensor& q, const Tensor& m) {
    want(q, at::kFloat, "q");
    want(m, at::kFloat, "m");
    TORCH_CHECK(q.dim() == 2 && m.dim() == 2 && q.size(1) == m.size(1), "xcorr shapes");
    c10::DeviceGuard g(q.device());
    Tensor out = at::empty({1}, q.options());
    Tensor ws = workspace(mlg_xcorr_workspace_bytes((int)q.size(0), (int)m.size(0), (int)q.size(1)), q);
    check_rc(mlg_xcorr_score(cp<float>(q), (int)q.size(0), cp<float>(m), (int)m.size(0), (int)q.size(1), ws.data_ptr(),
                             (size_t)ws.numel(), mp<float>(out), stream_of(q)),
             "mlg_xcorr_score");
    return out;
}

// -------------------------------------------------------------- SuperPoint
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> superpoint(const Tensor& frames, at::TensorList w,
                                                               double det_thr, int64_t max_kp, int64_t nms_radius,
                                                               int64_t border, bool with_bf16) {
    want(frames, at::kByte, "frames");
    TORCH_CHECK(frames.dim() == 4, "frames must be [B, H, W, C]");
    TORCH_CHECK(w.size() == 24, "superpoint weights: expected 24 tensors");
    mlg_sp_weights s = MLG_STRUCT_INIT(mlg_sp_weights);
    s.conv1a_w = cp<float>(w[0]);
    s.conv1a_b = cp<float>(w[1]);
    for (int i = 0; i < 11; ++i) {
        s.w[i] = cp<uint16_t>(w[2 + i]);
        s.b[i] = cp<float>(w[13 + i]);
    }
    const int64_t B = frames.size(0), H = frames.size(1), W = frames.size(2), C = frames.size(3);
    const size_t nbytes = mlg_superpoint_workspace_bytes((int)B, (int)H, (int)W);
    TORCH_CHECK(nbytes > 0, "SuperPoint needs H, W >= 16 (got ", H, "x", W, ")");
    c10::DeviceGuard g(frames.device());
    auto o = frames.options();
    Tensor kp = at::zeros({B, max_kp, 2}, o.dtype(at::kFloat)), sc = at::zeros({B, max_kp}, o.dtype(at::kFloat));
    Tensor ds = at::empty({B, max_kp, 256}, o.dtype(at::kFloat));
    Tensor db = with_bf16 ? at::empty({B, max_kp, 256}, o.dtype(at::kBFloat16)) : at::empty({0}, o.dtype(at::kBFloat16));
    Tensor cnt = at::empty({B}, o.dtype(at::kInt));
    Tensor ws = workspace(nbytes, frames);
    check_rc(mlg_superpoint(&s, cp<uint8_t>(frames), (int)B, (int)H, (int)W, (int)C, (long)(H * W * C), (float)det_thr,
                            (int)max_kp, (int)nms_radius, (int)border, ws.data_ptr(), (size_t)ws.numel(),
                            mp<float>(kp), mp<float>(sc), mp<float>(ds), with_bf16 ? mp<uint16_t>(db) : nullptr,
                            mp<int32_t>(cnt), stream_of(frames)),
             "mlg_superpoint");
    return {kp, sc, ds, db, cnt};
}

// ------------------------------------------------------------------ LoFTR
// weights: stem_w, stem_b, conv_w[21], conv_b[21] (empty = none), 8 coarse + 2 fine
// layers x (w, wmerge, w1, w2, ln1_g, ln1_b, ln2_g, ln2_b), down_w, down_b, merge_wf,
// merge_wc, merge_b (mlgate/loftr.py builds the list), optionally followed by the packed
// coarse tails (uint8 [mlg_loftr_tails_bytes()], loftr_pack_tails)
constexpr int kLoftrTensors = 2 + 2 * MLG_LOFTR_NCONV + 10 * 8 + 5;

mlg_loftr_weights loftr_weights(at::TensorList w) {
    TORCH_CHECK((int)w.size() == kLoftrTensors || (int)w.size() == kLoftrTensors + 1, "loftr weights: expected ",
                kLoftrTensors, " (+ 1 packed tails) tensors, got ", w.size());
    mlg_loftr_weights s = MLG_STRUCT_INIT(mlg_loftr_weights);
    int i = 0;
    s.stem_w = cp<float>(w[i++]);
    s.stem_b = cp<float>(w[i++]);
    for (int c = 0; c < MLG_LOFTR_NCONV; ++c) s.conv_w[c] = cp<uint16_t>(w[i++]);
    for (int c = 0; c < MLG_LOFTR_NCONV; ++c) s.conv_b[c] = cp<float>(w[i++]);
    for (int l = 0; l < 10; ++l) {
        mlg_loftr_layer& L = l < 8 ? s.coarse[l] : s.fine[l - 8];
        L.w = cp<uint16_t>(w[i++]);
        L.wmerge = cp<uint16_t>(w[i++]);
        L.w1 = cp<uint16_t>(w[i++]);
        L.w2 = cp<uint16_t>(w[i++]);
        L.ln1_g = cp<float>(w[i++]);
        L.ln1_b = cp<float>(w[i++]);
        L.ln2_g = cp<float>(w[i++]);
        L.ln2_b = cp<float>(w[i++]);
    }
    s.down_w = cp<uint16_t>(w[i++]);
    s.down_b = cp<float>(w[i++]);
    s.merge_wf = cp<uint16_t>(w[i++]);
    s.merge_wc = cp<uint16_t>(w[i++]);
    s.merge_b = cp<float>(w[i++]);
    if ((int)w.size() > kLoftrTensors) {
        const Tensor& t = w[i];
        TORCH_CHECK(t.scalar_type() == at::kByte && (size_t)t.numel() == mlg_loftr_tails_bytes() && t.is_contiguous(),
                    "loftr packed tails must be uint8 [", mlg_loftr_tails_bytes(), "] (loftr_pack_tails)");
        s.coarse_tails = t.data_ptr();
    }
    return s;
}

// one coarse encoder layer in place, fused or unfused tail (mlg_op_loftr_coarse_layer)
void loftr_coarse_layer(const Tensor& x, const Tensor& cat, at::TensorList w, int64_t layer, int64_t fused,
                        int64_t nseg, int64_t L) {
    want(x, at::kFloat, "x");
    want(cat, at::kBFloat16, "cat");
    TORCH_CHECK(x.numel() == 2 * nseg * L * 256 && cat.numel() == 2 * nseg * L * 512,
                "x must be [2 nseg L, 256], cat [2 nseg L, 512]");
    const mlg_loftr_weights s = loftr_weights(w);
    c10::DeviceGuard g(x.device());
    Tensor ws = workspace(mlg_op_loftr_coarse_layer_ws_bytes((int)nseg, (int)L), x);
    check_rc(mlg_op_loftr_coarse_layer(&s, (int)layer, (int)fused, mp<float>(x), mp<uint16_t>(cat), (int)nseg, (int)L,
                                       ws.data_ptr(), (size_t)ws.numel(), stream_of(x)),
             "mlg_op_loftr_coarse_layer");
}

// the coarse block-tail weights packed once for the fused kernel (mlg_loftr_pack_tails)
Tensor loftr_pack_tails(at::TensorList w) {
    TORCH_CHECK((int)w.size() == kLoftrTensors, "loftr weights: expected ", kLoftrTensors, " tensors");
    const mlg_loftr_weights s = loftr_weights(w);
    c10::DeviceGuard g(w[0].device());
    Tensor out = at::empty({(int64_t)mlg_loftr_tails_bytes()}, w[0].options().dtype(at::kByte));
    check_rc(mlg_loftr_pack_tails(&s, out.data_ptr(), stream_of(w[0])), "mlg_loftr_pack_tails");
    return out;
}

std::tuple<Tensor, Tensor> loftr_features(const Tensor& frames, at::TensorList w) {
    want(frames, at::kByte, "frames");
    TORCH_CHECK(frames.dim() == 4, "frames must be [B, H, W, C]");
    const mlg_loftr_weights s = loftr_weights(w);
    const int64_t B = frames.size(0), H = frames.size(1), W = frames.size(2), C = frames.size(3);
    const size_t nbytes = mlg_loftr_features_ws_bytes((int)B, (int)H, (int)W);
    TORCH_CHECK(nbytes > 0, "LoFTR needs H, W >= 32 (got ", H, "x", W, ")");
    c10::DeviceGuard g(frames.device());
    auto o = frames.options().dtype(at::kFloat);
    const int64_t H8 = H / 8 * 8, W8 = W / 8 * 8;
    Tensor coarse = at::empty({B, (H8 / 8) * (W8 / 8), 256}, o), fine = at::empty({B, (H8 / 2) * (W8 / 2), 128}, o);
    Tensor ws = workspace(nbytes, frames);
    check_rc(mlg_loftr_features(&s, cp<uint8_t>(frames), (int)B, (int)H, (int)W, (int)C, (long)(H * W * C),
                                ws.data_ptr(), (size_t)ws.numel(), mp<float>(coarse), mp<float>(fine),
                                stream_of(frames)),
             "mlg_loftr_features");
    return {coarse, fine};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> loftr_match(const Tensor& coarse, const Tensor& fine, const Tensor& pa,
                                                       const Tensor& pb, const Tensor& pe, at::TensorList w, int64_t H,
                                                       int64_t W) {
    want(coarse, at::kFloat, "coarse");
    want(fine, at::kFloat, "fine");
    want(pe, at::kFloat, "pe");
    want(pa, at::kInt, "pair_a", false);
    want(pb, at::kInt, "pair_b", false);
    const int64_t P = pa.numel(), F = coarse.size(0), L = (H / 8) * (W / 8);
    TORCH_CHECK(pb.numel() == P && P > 0, "pair lists must be non-empty and of equal length");
    TORCH_CHECK(coarse.dim() == 3 && coarse.size(1) == L && coarse.size(2) == 256, "coarse must be [F, H/8*W/8, 256]");
    TORCH_CHECK(fine.dim() == 3 && fine.size(0) == F && fine.size(1) == (H / 2) * (W / 2) && fine.size(2) == 128,
                "fine must be [F, H/2*W/2, 128]");
    TORCH_CHECK(pe.numel() == L * 256, "pe must be [H/8*W/8, 256]");
    const int32_t* a = pa.data_ptr<int32_t>();
    const int32_t* b = pb.data_ptr<int32_t>();
    for (int64_t p = 0; p < P; ++p)
        TORCH_CHECK(a[p] >= 0 && a[p] < F && b[p] >= 0 && b[p] < F, "pair ", p, " indexes a missing frame");
    const mlg_loftr_weights s = loftr_weights(w);
    const size_t nbytes = mlg_loftr_match_ws_bytes((int)P, (int)H, (int)W);
    TORCH_CHECK(nbytes > 0, "LoFTR needs H, W >= 32 and multiples of 8");
    c10::DeviceGuard g(coarse.device());
    auto o = coarse.options();
    Tensor counts = at::empty({P}, o.dtype(at::kInt));
    Tensor k0 = at::zeros({P, L, 2}, o), k1 = at::zeros({P, L, 2}, o), cf = at::zeros({P, L}, o);
    Tensor ws = workspace(nbytes, coarse);
    check_rc(mlg_loftr_match(&s, cp<float>(coarse), cp<float>(fine), (int)H, (int)W, a, b, (int)P, cp<float>(pe),
                             ws.data_ptr(), (size_t)ws.numel(), mp<int32_t>(counts), mp<float>(k0), mp<float>(k1),
                             mp<float>(cf), stream_of(coarse)),
             "mlg_loftr_match");
    return {counts, k0, k1, cf};
}

// --------------------------------------------------------------- SuperGlue
// weights: kenc_w[0..2], kenc_b[0..2], kenc_w4, kenc_b4, kenc_w5, kenc_b5, 18 layers x
// (Wqkv, bqkv, Wout, bout, Wf1, bf1, Wf2, bf2), Wfinal, bfinal; bin_score as a double
constexpr int kSgTensors = 6 + 4 + 18 * 8 + 2;

std::tuple<Tensor, Tensor, Tensor> superglue(const Tensor& kpts, const Tensor& scores, const Tensor& desc,
                                             const Tensor& counts, const Tensor& pair_a, const Tensor& pair_b,
                                             at::TensorList w, double bin_score, int64_t W, int64_t H, int64_t iters,
                                             double thr) {
    want(kpts, at::kFloat, "kpts");
    want(scores, at::kFloat, "scores");
    want(desc, at::kFloat, "desc");
    want(counts, at::kInt, "counts", false);
    want(pair_a, at::kInt, "pair_a", false);
    want(pair_b, at::kInt, "pair_b", false);
    TORCH_CHECK((int)w.size() == kSgTensors, "superglue weights: expected ", kSgTensors, " tensors");
    const int64_t F = kpts.size(0), kmax = kpts.size(1), P = pair_a.numel();
    TORCH_CHECK(kpts.dim() == 3 && kpts.size(2) == 2 && desc.dim() == 3 && desc.size(0) == F &&
                    desc.size(1) == kmax && desc.size(2) == 256 && scores.numel() == F * kmax,
                "kpts [F, kmax, 2] / scores [F, kmax] / desc [F, kmax, 256]");
    TORCH_CHECK(counts.numel() == F && pair_b.numel() == P && P > 0, "counts [F], pair_a / pair_b [P]");
    const int32_t* cn = cp<int32_t>(counts);
    for (int64_t f = 0; f < F; ++f) TORCH_CHECK(cn[f] >= 0 && cn[f] <= kmax, "counts out of range");
    mlg_sg_weights s = MLG_STRUCT_INIT(mlg_sg_weights);
    int i = 0;
    for (int l = 0; l < 3; ++l) s.kenc_w[l] = cp<float>(w[i++]);
    for (int l = 0; l < 3; ++l) s.kenc_b[l] = cp<float>(w[i++]);
    s.kenc_w4 = cp<uint16_t>(w[i++]);
    s.kenc_b4 = cp<float>(w[i++]);
    s.kenc_w5 = cp<uint16_t>(w[i++]);
    s.kenc_b5 = cp<float>(w[i++]);
    for (int l = 0; l < 18; ++l) {
        mlg_lg_block& b = s.layer[l];
        b.Wqkv = cp<uint16_t>(w[i++]); b.bqkv = cp<float>(w[i++]);
        b.Wout = cp<uint16_t>(w[i++]); b.bout = cp<float>(w[i++]);
        b.Wf1 = cp<uint16_t>(w[i++]); b.bf1 = cp<float>(w[i++]);
        b.Wf2 = cp<uint16_t>(w[i++]); b.bf2 = cp<float>(w[i++]);
    }
    s.Wfinal = cp<uint16_t>(w[i++]);
    s.bfinal = cp<float>(w[i++]);
    s.bin_score = (float)bin_score;
    const size_t nbytes = mlg_superglue_workspace_bytes((int)P, (int)kmax);
    c10::DeviceGuard g(kpts.device());
    auto o = kpts.options();
    Tensor m = at::empty({P, kmax, 2}, o.dtype(at::kInt)), sc = at::empty({P, kmax}, o.dtype(at::kFloat));
    Tensor n = at::empty({P}, o.dtype(at::kInt));
    Tensor ws = workspace(nbytes, kpts);
    check_rc(mlg_superglue(&s, cp<float>(kpts), cp<float>(scores), cp<float>(desc), cn, (int)F, (int)kmax, (int)W,
                           (int)H, cp<int32_t>(pair_a), cp<int32_t>(pair_b), (int)P, (int)iters, (float)thr,
                           ws.data_ptr(), (size_t)ws.numel(), mp<int32_t>(m), mp<float>(sc), mp<int32_t>(n),
                           stream_of(kpts)),
             "mlg_superglue");
    return {m, sc, n};
}

// CricaVPR.rerank_candidates at scale: feats f32 [F, L, D], query / cand int32 [P] -> scores f32 [P]
Tensor xcorr_batch(const Tensor& feats, const Tensor& query, const Tensor& cand) {
    want(feats, at::kFloat, "feats");
    want(query, at::kInt, "query");
    want(cand, at::kInt, "cand");
    TORCH_CHECK(feats.dim() == 3 && feats.size(2) % 4 == 0, "feats [F, L, D] with D % 4 == 0");
    TORCH_CHECK(query.numel() == cand.numel(), "query / cand [P]");
    const int64_t F = feats.size(0), L = feats.size(1), D = feats.size(2), P = query.numel();
    c10::DeviceGuard g(feats.device());
    Tensor out = at::empty({P}, feats.options());
    if (P == 0) return out;
    Tensor ws = workspace(mlg_xcorr_batch_workspace_bytes((int)F, (int)L, (int)D, (int)P), feats);
    check_rc(mlg_xcorr_batch(cp<float>(feats), (int)F, (int)L, (int)D, cp<int32_t>(query), cp<int32_t>(cand), (int)P,
                             ws.data_ptr(), (size_t)ws.numel(), mp<float>(out), stream_of(feats)),
             "mlg_xcorr_batch");
    return out;
}

// --------------------------------------------------------------- LightGlue
constexpr int kLgTensors = 1 + 9 * 10 * 2 + 9 * 4 + 8 * 2 + 1;

std::tuple<Tensor, Tensor, Tensor, Tensor> lightglue(const Tensor& kpts, const Tensor& desc, const Tensor& counts,
                                                     const Tensor& pair_a, const Tensor& pair_b, at::TensorList w,
                                                     double depth_conf, double width_conf, double filter_thr,
                                                     int64_t pruning_min) {
    want(kpts, at::kFloat, "kpts");
    want(desc, at::kFloat, "desc");
    want(counts, at::kInt, "counts", false);
    want(pair_a, at::kInt, "pair_a", false);
    want(pair_b, at::kInt, "pair_b", false);
    TORCH_CHECK((int)w.size() == kLgTensors, "lightglue weights: expected ", kLgTensors, " tensors");
    const int64_t F = kpts.size(0), kmax = kpts.size(1), P = pair_a.numel();
    TORCH_CHECK(kpts.dim() == 3 && kpts.size(2) == 2 && desc.dim() == 3 && desc.size(0) == F &&
                    desc.size(1) == kmax && desc.size(2) == 256, "kpts [F, kmax, 2] / desc [F, kmax, 256]");
    TORCH_CHECK(counts.numel() == F && pair_b.numel() == P, "counts [F], pair_a / pair_b [P]");
    const int32_t* pa = cp<int32_t>(pair_a);
    const int32_t* pb = cp<int32_t>(pair_b);
    const int32_t* cn = cp<int32_t>(counts);
    for (int64_t p = 0; p < P; ++p)
        TORCH_CHECK(pa[p] >= 0 && pa[p] < F && pb[p] >= 0 && pb[p] < F, "pair frame index out of range");
    for (int64_t f = 0; f < F; ++f) TORCH_CHECK(cn[f] >= 0 && cn[f] <= kmax, "counts out of range");
    mlg_lg_weights s = MLG_STRUCT_INIT(mlg_lg_weights);
    int i = 0;
    s.Wr = cp<float>(w[i++]);
    for (mlg_lg_block* blocks : {s.self, s.cross})
        for (int l = 0; l < 9; ++l) {
            mlg_lg_block& b = blocks[l];
            b.Wqkv = cp<uint16_t>(w[i++]); b.bqkv = cp<float>(w[i++]);
            b.Wout = cp<uint16_t>(w[i++]); b.bout = cp<float>(w[i++]);
            b.Wf1 = cp<uint16_t>(w[i++]); b.bf1 = cp<float>(w[i++]);
            b.ln_g = cp<float>(w[i++]); b.ln_b = cp<float>(w[i++]);
            b.Wf2 = cp<uint16_t>(w[i++]); b.bf2 = cp<float>(w[i++]);
        }
    for (int l = 0; l < 9; ++l) s.Wfinal[l] = cp<uint16_t>(w[i++]);
    for (int l = 0; l < 9; ++l) s.bfinal[l] = cp<float>(w[i++]);
    for (int l = 0; l < 9; ++l) s.wmatch[l] = cp<float>(w[i++]);
    for (int l = 0; l < 9; ++l) s.bmatch[l] = cp<float>(w[i++]);
    for (int l = 0; l < 8; ++l) s.wconf[l] = cp<float>(w[i++]);
    for (int l = 0; l < 8; ++l) s.bconf[l] = cp<float>(w[i++]);
    s.ones = cp<float>(w[i++]);
    const size_t nbytes = mlg_lightglue_workspace_bytes((int)P, (int)kmax);
    TORCH_CHECK(nbytes > 0, "LightGlue supports up to 2048 keypoints per image (got ", kmax, ")");
    c10::DeviceGuard g(kpts.device());
    auto o = kpts.options();
    Tensor m = at::empty({P, kmax, 2}, o.dtype(at::kInt)), sc = at::empty({P, kmax}, o.dtype(at::kFloat));
    Tensor n = at::empty({P}, o.dtype(at::kInt));
    Tensor stop = at::zeros({P}, counts.options());
    if (P == 0) return {m, sc, n, stop};
    Tensor ws = workspace(nbytes, kpts);
    check_rc(mlg_lightglue(&s, cp<float>(kpts), cp<float>(desc), cn, (int)F, (int)kmax, pa, pb, (int)P,
                           (float)depth_conf, (float)width_conf, (float)filter_thr, (int)pruning_min, ws.data_ptr(),
                           (size_t)ws.numel(), mp<int32_t>(m), mp<float>(sc), mp<int32_t>(n), mp<int32_t>(stop),
                           stream_of(kpts)),
             "mlg_lightglue");
    return {m, sc, n, stop};
}

std::tuple<Tensor, Tensor, Tensor> lg_orient(const Tensor& m, const Tensor& sc, const Tensor& n, const Tensor& rows,
                                             const Tensor& swap) {
    want(m, at::kInt, "matches");
    want(sc, at::kFloat, "scores");
    want(n, at::kInt, "num_matches");
    want(rows, at::kInt, "rows");
    want(swap, at::kByte, "swap");
    TORCH_CHECK(m.dim() == 3 && m.size(2) == 2 && sc.size(0) == m.size(0) && n.numel() == m.size(0),
                "matches [R, kmax, 2], scores [R, kmax], num [R]");
    TORCH_CHECK(rows.numel() == swap.numel(), "rows / swap sizes differ");
    const int64_t P = rows.numel(), kmax = m.size(1);
    c10::DeviceGuard g(m.device());
    Tensor mo = at::empty({P, kmax, 2}, m.options()), so = at::empty({P, kmax}, sc.options());
    Tensor no = at::empty({P}, n.options());
    check_rc(mlg_lg_orient_matches(cp<int32_t>(m), cp<float>(sc), cp<int32_t>(n), cp<int32_t>(rows),
                                   cp<uint8_t>(swap), (int)P, (int)kmax, mp<int32_t>(mo), mp<float>(so),
                                   mp<int32_t>(no), stream_of(m)),
             "mlg_lg_orient_matches");
    return {mo, so, no};
}

// ------------------------------------------------------------------ RANSAC
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> ransac_epipolar(const Tensor& k1, const Tensor& k2,
                                                                   const Tensor& offs, const c10::optional<Tensor>& K,
                                                                   int64_t k_stride, double thr, int64_t hypotheses,
                                                                   int64_t seed, bool with_pose) {
    want(k1, at::kFloat, "k1");
    want(k2, at::kFloat, "k2");
    want(offs, at::kInt, "offs");
    const bool has_k = K.has_value() && K->defined();
    if (has_k) want(*K, at::kDouble, "K");
    const int64_t P = offs.numel() - 1, S = k1.size(0);
    TORCH_CHECK(P >= 1 && k1.dim() == 2 && k1.size(1) == 2 && k2.sizes() == k1.sizes(), "ransac shapes");
    TORCH_CHECK(!has_k || K->numel() >= 9 + (P - 1) * k_stride, "K too small for the pairs");
    const size_t nbytes = mlg_ransac_workspace_bytes((int)P, (long)S, (int)hypotheses);
    TORCH_CHECK(nbytes > 0, "bad RANSAC shape");
    c10::DeviceGuard g(k1.device());
    auto o = k1.options();
    Tensor model = at::empty({P, 9}, o.dtype(at::kDouble)), mask = at::empty({std::max<int64_t>(S, 1)}, o.dtype(at::kByte));
    Tensor inl = at::empty({P}, o.dtype(at::kInt)), status = at::empty({P}, o.dtype(at::kInt));
    Tensor pose = (with_pose && has_k) ? at::empty({P, 16}, o.dtype(at::kDouble)) : at::empty({0}, o.dtype(at::kDouble));
    Tensor ws = workspace(nbytes, k1);
    check_rc(mlg_ransac_epipolar(cp<float>(k1), cp<float>(k2), cp<int32_t>(offs), (int)P, (long)S,
                                 has_k ? cp<double>(*K) : nullptr, (int)k_stride, thr, (int)hypotheses, (uint64_t)seed,
                                 ws.data_ptr(), (size_t)ws.numel(), mp<double>(model), mp<uint8_t>(mask),
                                 mp<int32_t>(inl), pose.numel() ? mp<double>(pose) : nullptr, mp<int32_t>(status),
                                 stream_of(k1)),
             "mlg_ransac_epipolar");
    return {model, mask.narrow(0, 0, S), inl, pose, status};
}

Tensor recover_pose(const Tensor& k1, const Tensor& k2, const Tensor& offs, const Tensor& K, int64_t k_stride,
                    const Tensor& E, const Tensor& mask) {
    want(k1, at::kFloat, "k1");
    want(k2, at::kFloat, "k2");
    want(offs, at::kInt, "offs");
    want(K, at::kDouble, "K");
    want(E, at::kDouble, "E");
    want(mask, at::kByte, "mask");
    const int64_t P = offs.numel() - 1;
    TORCH_CHECK(P >= 1 && E.numel() == 9 * P, "E must be [P, 9]");
    c10::DeviceGuard g(k1.device());
    Tensor pose = at::empty({P, 16}, k1.options().dtype(at::kDouble));
    check_rc(mlg_recover_pose(cp<float>(k1), cp<float>(k2), cp<int32_t>(offs), (int)P, cp<double>(K), (int)k_stride,
                              cp<double>(E), cp<uint8_t>(mask), mp<double>(pose), stream_of(k1)),
             "mlg_recover_pose");
    return pose;
}

// --------------------------------------------------------------- ResNet-50
Tensor resnet50(const Tensor& frames, at::TensorList w, int64_t descriptor_dim) {
    want(frames, at::kByte, "frames");
    TORCH_CHECK(frames.dim() == 4, "frames must be [B, H, W, C]");
    TORCH_CHECK(w.size() == 2 + 16 * 8, "resnet50 weights: expected 130 tensors");
    mlg_rn_weights s = MLG_STRUCT_INIT(mlg_rn_weights);
    s.stem_w = cp<float>(w[0]);
    s.stem_b = cp<float>(w[1]);
    for (int b = 0; b < 16; ++b) {
        const Tensor* t = &w[2 + 8 * b];
        mlg_rn_block& o = s.blocks[b];
        o.w1 = cp<uint16_t>(t[0]); o.b1 = cp<float>(t[1]);
        o.w2 = cp<uint16_t>(t[2]); o.b2 = cp<float>(t[3]);
        o.w3 = cp<uint16_t>(t[4]); o.b3 = cp<float>(t[5]);
        o.wd = cp<uint16_t>(t[6]); o.bd = cp<float>(t[7]);
    }
    const int64_t B = frames.size(0), H = frames.size(1), W = frames.size(2), C = frames.size(3);
    c10::DeviceGuard g(frames.device());
    Tensor out = at::empty({B, descriptor_dim}, frames.options().dtype(at::kFloat));
    Tensor ws = workspace(mlg_resnet50_workspace_bytes((int)B, (int)H, (int)W), frames);
    check_rc(mlg_resnet50_forward(&s, cp<uint8_t>(frames), (int)B, (int)H, (int)W, (int)C, (long)(H * W * C),
                                  (int)descriptor_dim, ws.data_ptr(), (size_t)ws.numel(), mp<float>(out),
                                  stream_of(frames)),
             "mlg_resnet50_forward");
    return out;
}

Tensor pillow_resize_224(const Tensor& frames) {
    want(frames, at::kByte, "frames");
    const int64_t B = frames.size(0), H = frames.size(1), W = frames.size(2), C = frames.size(3);
    c10::DeviceGuard g(frames.device());
    Tensor out = at::empty({B, 224, 224, 3}, frames.options());
    Tensor ws = workspace(mlg_resnet50_workspace_bytes((int)B, (int)H, (int)W), frames);
    check_rc(mlg_op_pillow_resize_224(cp<uint8_t>(frames), (int)B, (int)H, (int)W, (int)C, (long)(H * W * C),
                                      ws.data_ptr(), (size_t)ws.numel(), mp<uint8_t>(out), stream_of(frames)),
             "mlg_op_pillow_resize_224");
    return out;
}

// ---------------------------------------------------- LiDAR plane RANSAC
std::tuple<Tensor, Tensor, Tensor> plane_ransac(const Tensor& pts, const Tensor& offsets, int64_t iterations,
                                                int64_t seed, double threshold) {
    want(pts, at::kFloat, "pts");
    want(offsets, at::kInt, "offsets");
    const int64_t S = offsets.numel() - 1;
    TORCH_CHECK(S >= 1 && iterations >= 1, "plane_ransac shapes");
    c10::DeviceGuard g(pts.device());
    auto o = pts.options();
    Tensor plane = at::empty({S, 4}, o.dtype(at::kDouble)), ratio = at::empty({S}, o.dtype(at::kDouble));
    Tensor inl = at::empty({S}, o.dtype(at::kInt));
    Tensor ws = workspace(mlg_plane_ransac_workspace_bytes((int)S, (int)iterations), pts);
    check_rc(mlg_plane_ransac(cp<float>(pts), cp<int32_t>(offsets), (int)S, (int)iterations, (uint64_t)seed, threshold,
                              ws.data_ptr(), (size_t)ws.numel(), mp<double>(plane), mp<double>(ratio),
                              mp<int32_t>(inl), stream_of(pts)),
             "mlg_plane_ransac");
    return {plane, ratio, inl};
}

// ------------------------------------------------- trajectory proximity
// count + emit in one op; reads the candidate count back (output size is data-dependent)
std::tuple<Tensor, Tensor, Tensor, Tensor> proximity(const Tensor& pos, const c10::optional<Tensor>& floor,
                                                     int64_t row0, int64_t nrows, double radius, int64_t min_gap,
                                                     bool strict) {
    want(pos, at::kDouble, "pos");
    const bool hf = floor.has_value() && floor->defined();
    if (hf) want(*floor, at::kLong, "floor");
    const int64_t N = pos.size(0);
    TORCH_CHECK(pos.dim() == 2 && pos.size(1) == 3 && row0 >= 0 && nrows >= 0 && row0 + nrows <= N,
                "proximity shapes");
    c10::DeviceGuard g(pos.device());
    auto o = pos.options();
    const size_t nbytes = mlg_proximity_workspace_bytes((int)N, (int)nrows);
    TORCH_CHECK(nbytes > 0, "proximity search supports up to 65536 poses");
    Tensor ws = workspace(nbytes, pos);
    Tensor totals = at::zeros({2}, o.dtype(at::kLong));
    const int64_t* fl = hf ? cp<int64_t>(*floor) : nullptr;
    check_rc(mlg_proximity_count(cp<double>(pos), fl, (int)N, (int)row0, (int)nrows, radius, (int)min_gap,
                                 strict ? 1 : 0, ws.data_ptr(), (size_t)ws.numel(), mp<long long>(totals),
                                 stream_of(pos)),
             "mlg_proximity_count");
    const int64_t n = totals.cpu().data_ptr<int64_t>()[0];
    Tensor pairs = at::empty({n, 2}, o.dtype(at::kInt)), dist = at::empty({n}, o.dtype(at::kDouble));
    Tensor valid = at::empty({n}, o.dtype(at::kByte));
    if (n > 0)
        check_rc(mlg_proximity_emit(cp<double>(pos), fl, (int)N, (int)row0, (int)nrows, radius, (int)min_gap,
                                    strict ? 1 : 0, ws.data_ptr(), (size_t)ws.numel(), mp<int32_t>(pairs),
                                    mp<double>(dist), mp<uint8_t>(valid), stream_of(pos)),
                 "mlg_proximity_emit");
    return {pairs, dist, valid, totals};
}

// ------------------------------------------------------------- profiling
int64_t prof_enable(int64_t mask) { return mlg_prof_enable((int)mask); }
int64_t prof_reset() { return mlg_prof_reset(); }
std::tuple<double, int64_t, double> prof_read(int64_t slot) {
    double ms = 0.0, work = 0.0;
    long n = 0;
    check_rc(mlg_prof_read((int)slot, &ms, &n), "mlg_prof_read");
    check_rc(mlg_prof_read_work((int)slot, &work), "mlg_prof_read_work");
    return {ms, (int64_t)n, work};
}


// ------------------------------------------------------------------ ORB fallback
// iparams: int32 [57] = level_w[8], level_h[8], level_features[8], level_vec_end[8],
// umax[16], gauss[7], fast_threshold, edge_threshold; scales: float32 [8] (host tensors)
mlg_orb_params orb_params(const Tensor& ip, const Tensor& fp) {
    want(ip, at::kInt, "orb iparams", false);
    want(fp, at::kFloat, "orb fparams", false);
    TORCH_CHECK(ip.numel() == 42 && fp.numel() == MLG_ORB_LEVELS + 7,
                "orb params: expected 42 ints and 8 scales + 7 Gaussian taps");
    const int32_t* v = ip.data_ptr<int32_t>();
    const float* f = fp.data_ptr<float>();
    mlg_orb_params p = MLG_STRUCT_INIT(mlg_orb_params);
    for (int l = 0; l < MLG_ORB_LEVELS; ++l) {
        p.level_w[l] = v[l];
        p.level_h[l] = v[8 + l];
        p.level_features[l] = v[16 + l];
        p.level_scale[l] = f[l];
    }
    for (int i = 0; i < 16; ++i) p.umax[i] = v[24 + i];
    for (int i = 0; i < 7; ++i) p.gauss[i] = f[MLG_ORB_LEVELS + i];
    p.fast_threshold = v[40];
    p.edge_threshold = v[41];
    return p;
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> orb_detect(Tensor frames, Tensor pattern, Tensor iparams,
                                                                      Tensor scales, int64_t max_kp) {
    want(frames, at::kByte, "frames");
    want(pattern, at::kShort, "pattern");
    TORCH_CHECK(frames.dim() == 4, "frames: [F, H, W, C] uint8");
    TORCH_CHECK(pattern.numel() == 1024, "pattern: 256 pairs x 2 points x (x, y)");
    const c10::DeviceGuard guard(frames.device());
    const mlg_orb_params p = orb_params(iparams, scales);
    const int F = (int)frames.size(0), H = (int)frames.size(1), W = (int)frames.size(2), C = (int)frames.size(3);
    const size_t wsb = mlg_orb_workspace_bytes(&p, F, H, W, (int)max_kp);
    TORCH_CHECK(wsb > 0, "orb_detect: invalid geometry");
    Tensor ws = workspace(wsb, frames);
    auto o = frames.options();
    Tensor kp = at::empty({F, max_kp, 2}, o.dtype(at::kFloat)), resp = at::empty({F, max_kp}, o.dtype(at::kFloat));
    Tensor ang = at::empty({F, max_kp}, o.dtype(at::kFloat)), lev = at::empty({F, max_kp}, o.dtype(at::kInt));
    Tensor desc = at::zeros({F, max_kp, 32}, o), cnt = at::empty({F}, o.dtype(at::kInt));
    check_rc(mlg_orb_detect(&p, cp<int16_t>(pattern), cp<uint8_t>(frames), (long)H * W * C, F, H, W, C, (int)max_kp,
                            mp<void>(ws), wsb, mp<float>(kp), mp<float>(resp), mp<float>(ang), mp<int32_t>(lev),
                            mp<uint8_t>(desc), mp<int32_t>(cnt), stream_of(frames)),
             "mlg_orb_detect");
    return {kp, resp, ang, lev, desc, cnt};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> orb_match(Tensor desc, Tensor counts, Tensor pair_a, Tensor pair_b) {
    want(desc, at::kByte, "descriptors");
    want(counts, at::kInt, "counts");
    want(pair_a, at::kInt, "pair_a");
    want(pair_b, at::kInt, "pair_b");
    TORCH_CHECK(desc.dim() == 3 && desc.size(2) == 32, "descriptors: [F, max_kp, 32]");
    const c10::DeviceGuard guard(desc.device());
    const int P = (int)pair_a.numel(), K = (int)desc.size(1);
    TORCH_CHECK(pair_b.numel() == P, "pair_a / pair_b sizes differ");
    auto o = desc.options().dtype(at::kInt);
    Tensor q = at::empty({P, K}, o), t = at::empty({P, K}, o), d = at::empty({P, K}, o), n = at::zeros({P}, o);
    if (P == 0) return {q, t, d, n};
    const size_t wsb = mlg_orb_match_workspace_bytes(P, K);
    Tensor ws = workspace(wsb, desc);
    check_rc(mlg_orb_match(cp<uint8_t>(desc), cp<int32_t>(counts), K, cp<int32_t>(pair_a), cp<int32_t>(pair_b), P,
                           mp<void>(ws), wsb, mp<int32_t>(q), mp<int32_t>(t), mp<int32_t>(d), mp<int32_t>(n),
                           stream_of(desc)),
             "mlg_orb_match");
    return {q, t, d, n};
}

// ------------------------------------------------------------ keyframe ingestion
// Host ops (CPU key): the decoders write a caller-owned host tensor, normally a pinned
// staging buffer that mlgate.ingest uploads on a side stream.
Tensor png_load_into(std::vector<std::string> paths, Tensor out, int64_t H, int64_t W, int64_t threads) {
    want(out, at::kByte, "out", false);
    const int64_t n = (int64_t)paths.size();
    TORCH_CHECK(out.numel() >= n * H * W * 3, "out: needs ", n * H * W * 3, " bytes, has ", out.numel());
    std::vector<const char*> cps(paths.size());
    for (size_t i = 0; i < paths.size(); ++i) cps[i] = paths[i].c_str();
    Tensor status = at::zeros({n}, at::TensorOptions().dtype(at::kInt));
    check_rc(mlg_png_load_bgr(cps.data(), (int)n, mp<uint8_t>(out), (int)H, (int)W, (int)threads,
                              mp<int32_t>(status)), "mlg_png_load_bgr");
    return status;
}

std::tuple<Tensor, Tensor> png_decode(std::vector<Tensor> blobs, int64_t H, int64_t W, int64_t threads) {
    const int64_t n = (int64_t)blobs.size();
    std::vector<const uint8_t*> ptrs(n);
    std::vector<size_t> lens(n);
    for (int64_t i = 0; i < n; ++i) {
        want(blobs[i], at::kByte, "blob", false);
        ptrs[i] = cp<uint8_t>(blobs[i]);
        lens[i] = (size_t)blobs[i].numel();
    }
    Tensor out = at::zeros({n, H, W, 3}, at::TensorOptions().dtype(at::kByte));
    Tensor status = at::zeros({n}, at::TensorOptions().dtype(at::kInt));
    check_rc(mlg_png_decode_bgr(ptrs.data(), lens.data(), (int)n, mp<uint8_t>(out), (int)H, (int)W, (int)threads,
                                mp<int32_t>(status)), "mlg_png_decode_bgr");
    return {out, status};
}

}  // namespace

TORCH_LIBRARY(mlgate, m) {
    m.def("vit_forward_into(Tensor frames, Tensor[] weights, int image_size, int flags, int max_batch, "
          "Tensor(a!) desc, Tensor(b!)? local) -> ()");
    m.def("salad_forward(Tensor frames, Tensor[] weights, Tensor[] salad, float dust_bin, int image_size, "
          "int max_batch) -> Tensor");
    m.def("knn_gate(Tensor desc, Tensor t, Tensor floor, Tensor has_floor, float min_gap, float thr, int k, "
          "bool gating, int q0, int Q, Tensor(a!)? totals) -> (Tensor, Tensor, Tensor, Tensor)");
    m.def("knn_query(Tensor db, Tensor q, Tensor t_db, Tensor t_q, float min_gap, int k) -> (Tensor, Tensor, Tensor)");
    m.def("row_normalize(Tensor X) -> Tensor");
    m.def("similarity(Tensor A, Tensor B) -> Tensor");
    m.def("xcorr_score(Tensor q, Tensor m) -> Tensor");
    m.def("xcorr_batch(Tensor feats, Tensor query, Tensor cand) -> Tensor");
    m.def("superpoint(Tensor frames, Tensor[] weights, float detection_threshold, int max_keypoints, "
          "int nms_radius, int remove_borders, bool with_bf16) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
    m.def("lightglue(Tensor kpts, Tensor desc, Tensor counts, Tensor pair_a, Tensor pair_b, Tensor[] weights, "
          "float depth_confidence, float width_confidence, float filter_threshold, int pruning_min_kpts) "
          "-> (Tensor, Tensor, Tensor, Tensor)");
    m.def("ransac_epipolar(Tensor k1, Tensor k2, Tensor offsets, Tensor? K, int k_stride, float threshold, "
          "int hypotheses, int seed, bool with_pose) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
    m.def("recover_pose(Tensor k1, Tensor k2, Tensor offsets, Tensor K, int k_stride, Tensor E, Tensor mask) -> Tensor");
    m.def("resnet50(Tensor frames, Tensor[] weights, int descriptor_dim) -> Tensor");
    m.def("loftr_features(Tensor frames, Tensor[] weights) -> (Tensor, Tensor)");
    m.def("loftr_pack_tails(Tensor[] weights) -> Tensor");
    m.def("loftr_coarse_layer(Tensor(a!) x, Tensor(b!) cat, Tensor[] weights, int layer, int fused, int nseg, int L) -> ()");
    m.def("superglue(Tensor kpts, Tensor scores, Tensor desc, Tensor counts, Tensor pair_a, Tensor pair_b, "
          "Tensor[] weights, float bin_score, int W, int H, int iters, float threshold) -> (Tensor, Tensor, Tensor)");
    m.def("loftr_match(Tensor coarse, Tensor fine, Tensor pair_a, Tensor pair_b, Tensor pe, Tensor[] weights, int H, "
          "int W) -> (Tensor, Tensor, Tensor, Tensor)");
    m.def("pillow_resize_224(Tensor frames) -> Tensor");
    m.def("plane_ransac(Tensor pts, Tensor offsets, int iterations, int seed, float threshold) "
          "-> (Tensor, Tensor, Tensor)");
    m.def("proximity(Tensor pos, Tensor? floor, int row0, int nrows, float radius, int min_gap, bool strict) "
          "-> (Tensor, Tensor, Tensor, Tensor)");
    m.def("lg_orient(Tensor m, Tensor sc, Tensor n, Tensor rows, Tensor swap) -> (Tensor, Tensor, Tensor)");
    m.def("orb_detect(Tensor frames, Tensor pattern, Tensor iparams, Tensor scales, int max_kp) "
          "-> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
    m.def("orb_match(Tensor desc, Tensor counts, Tensor pair_a, Tensor pair_b) -> (Tensor, Tensor, Tensor, Tensor)");
    m.def("png_load_into(str[] paths, Tensor(a!) out, int H, int W, int threads) -> Tensor");
    m.def("png_decode(Tensor[] blobs, int H, int W, int threads) -> (Tensor, Tensor)");
    m.def("prof_enable(int mask) -> int");
    m.def("prof_reset() -> int");
    m.def("prof_read(int slot) -> (float, int, float)");
}

TORCH_LIBRARY_IMPL(mlgate, CUDA, m) {
    m.impl("vit_forward_into", &vit_forward_into);
    m.impl("salad_forward", &salad_forward);
    m.impl("knn_gate", &knn_gate);
    m.impl("knn_query", &knn_query);
    m.impl("row_normalize", &row_normalize);
    m.impl("similarity", &similarity);
    m.impl("xcorr_score", &xcorr_score);
    m.impl("xcorr_batch", &xcorr_batch);
    m.impl("superpoint", &superpoint);
    m.impl("lightglue", &lightglue);
    m.impl("ransac_epipolar", &ransac_epipolar);
    m.impl("recover_pose", &recover_pose);
    m.impl("resnet50", &resnet50);
    m.impl("loftr_features", &loftr_features);
    m.impl("loftr_pack_tails", &loftr_pack_tails);
    m.impl("loftr_coarse_layer", &loftr_coarse_layer);
    m.impl("superglue", &superglue);
    m.impl("loftr_match", &loftr_match);
    m.impl("pillow_resize_224", &pillow_resize_224);
    m.impl("plane_ransac", &plane_ransac);
    m.impl("proximity", &proximity);
    m.impl("lg_orient", &lg_orient);
    m.impl("orb_detect", &orb_detect);
    m.impl("orb_match", &orb_match);
}

TORCH_LIBRARY_IMPL(mlgate, CPU, m) {
    m.impl("png_load_into", &png_load_into);
    m.impl("png_decode", &png_decode);
}

TORCH_LIBRARY_IMPL(mlgate, CompositeExplicitAutograd, m) {
    m.impl("prof_enable", &prof_enable);
    m.impl("prof_reset", &prof_reset);
    m.impl("prof_read", &prof_read);
}
