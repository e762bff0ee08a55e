"""Oracle for CricaVPR local-feature cross-correlation (test infrastructure only).

Restates CricaVPR.compute_cross_correlation_score / rerank_candidates
(place_recognition.py:669-757) in float32 torch on the CPU: squeeze the batch dim,
row-normalise with +1e-8, C = q m^T, score = sqrt(mean(rowmax C) * mean(colmax C));
rerank: 0.5 * global + 0.5 * cross (global only when a feature set is not cached),
stable sort by combined score descending, keep top_k.
"""
import numpy as np
import torch


def xcorr_score(qf, mf):
    q = torch.from_numpy(np.asarray(qf, dtype=np.float32)).float()
    m = torch.from_numpy(np.asarray(mf, dtype=np.float32)).float()
    if q.dim() == 3:
        q = q.squeeze(0)
    if m.dim() == 3:
        m = m.squeeze(0)
    q = q / (q.norm(dim=-1, keepdim=True) + 1e-8)
    m = m / (m.norm(dim=-1, keepdim=True) + 1e-8)
    c = torch.mm(q, m.t())
    return float((c.max(dim=1)[0].mean() * c.max(dim=0)[0].mean()).sqrt())


def rerank(cache, query_idx, candidates, top_k=5, use_reranking=True):
    if not use_reranking or query_idx not in cache:
        return list(candidates[:top_k])
    out = []
    for j, g in candidates:
        out.append((j, 0.5 * g + 0.5 * xcorr_score(cache[query_idx], cache[j]) if j in cache else g))
    out.sort(key=lambda x: x[1], reverse=True)
    return out[:top_k]
