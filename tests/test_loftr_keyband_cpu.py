"""The LoFTR dual-softmax passes (csrc/loftr.hip k_lf_rowbest / k_lf_colmaxpart) find the
row argmax / column max of conf = softmax(sim, 1) * softmax(sim, 2) without evaluating
conf everywhere: conf_ij is proportional to exp(2 x_ij - rkey_i - ckey_j) (rkey = rmax +
log rsum, ckey = cmax + log csum), so only cells whose f32 key lies within
1e-3 + 1e-5 |key| of the best key get the exact conf.  This restates both searches in
float32 numpy on seeded similarity matrices -- wide and narrow value ranges, planted
exact and near ties -- and requires the banded result to equal the exhaustive one (the
argument the kernels rely on; the kernels themselves are GPU-tested end to end in
tests/test_loftr_gpu.py)."""
import numpy as np
import pytest

F = np.float32


def _stats(x, axis):
    m = x.max(axis=axis, keepdims=True)
    z = np.exp(x - m).sum(axis=axis, keepdims=True, dtype=F)
    return m.astype(F), z.astype(F)


def _conf(x, rm, rz, cm, cz):
    return (np.exp(x - cm) / cz) * (np.exp(x - rm) / rz)


def _band(k):
    return F(1e-3) + F(1e-5) * np.abs(k)


@pytest.mark.parametrize("seed,scale,n,m", [(0, 1.0, 300, 280), (1, 10.0, 257, 311), (2, 40.0, 200, 200),
                                            (3, 0.01, 128, 140), (4, 25.0, 64, 400)])
def test_banded_argmax_equals_exhaustive(seed, scale, n, m):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, m)) * scale).astype(F)
    # planted exact ties and near ties (a few ulps apart) in some rows / columns
    for i in range(0, n, 7):
        j = rng.integers(0, m - 1)
        x[i, j + 1] = x[i, j]
        x[i, (j + 3) % m] = np.nextafter(x[i, j], F(np.inf))
    rm, rz = _stats(x, 1)
    cm, cz = _stats(x, 0)
    conf = _conf(x, rm, rz, cm, cz).astype(F)
    rkey = (rm + np.log(rz)).astype(F)
    ckey = (cm + np.log(cz)).astype(F)
    key_r = (F(2) * x - ckey).astype(F)  # row search: per-column key
    key_c = (F(2) * x - rkey).astype(F)  # column search: per-row key
    # rows: max value, first index on ties
    for i in range(n):
        best = conf[i].max()
        want = int(np.flatnonzero(conf[i] == best)[0])
        kb = key_r[i].max()
        cand = np.flatnonzero(key_r[i] >= kb - _band(kb))
        got = int(cand[np.argmax(conf[i, cand])])  # argmax: first of the maxima in order
        assert conf[i, got] == best and got == want, (i, got, want)
    # columns: the exact max value
    for j in range(m):
        kb = key_c[:, j].max()
        cand = np.flatnonzero(key_c[:, j] >= kb - _band(kb))
        assert conf[cand, j].max() == conf[:, j].max(), j
