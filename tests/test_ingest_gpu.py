"""Keyframe ingestion on the GPU: PNG files -> HBM -> CricaVPR database.

process_image_sequence (place_recognition.py:936-991) is checked against the
reference's own loop run through the drop-in API: every frame decoded from its PNG,
add_image one at a time, find_loop_closures(enable_floor_gating=True).  The native
loader + device batches must give the same database (descriptors within 1e-6), the
same matches and the reference's warnings for a corrupt file and a count mismatch.
"""
import warnings

import numpy as np
import pytest
import torch

PIL = pytest.importorskip("PIL.Image")

import mlgate  # noqa: E402
from mlgate import ingest, synthetic  # noqa: E402
from mlgate.vpr import process_image_sequence  # noqa: E402

pytestmark = pytest.mark.gpu


def _write(tmp_path, frames, t):
    paths = []
    for f, ti in zip(frames, t):
        p = tmp_path / f"{ti:.6f}.png"       # bag_utils.extract_images' file name
        PIL.fromarray(f[..., ::-1]).save(p)  # cv2.imwrite stores BGR arrays as RGB PNG
        paths.append(p)
    return paths


def test_keyframe_stream_uploads_exact_frames(dev, tmp_path):
    seq = synthetic.make_sequence(10, places=4, seed=3)
    frames = synthetic.frames_host(seq, h=96, w=128)
    paths = _write(tmp_path, frames, seq.t)
    got = []
    for idx, fr in ingest.KeyframeStream(paths, device="cuda", batch=4):
        assert fr.device.type == "cuda" and fr.dtype == torch.uint8
        got.extend(zip(idx, fr.cpu().numpy()))
    assert [i for i, _ in got] == list(range(10))
    for i, f in got:
        assert np.array_equal(f, frames[i])


def test_process_image_sequence_matches_reference_loop(dev, tmp_path):
    n = 40
    seq = synthetic.make_sequence(n, places=6, seed=11)
    frames = synthetic.frames_host(seq)
    t = 100.0 + seq.t * 15.0  # spread so min_time_gap 10 s admits revisits
    floors = seq.floor_gt
    _write(tmp_path, frames, t)
    (tmp_path / "zzzz.png").write_bytes(b"\x89PNG\r\n\x1a\n broken")  # sorts last: imread -> None
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        spr, matches = process_image_sequence(tmp_path, np.append(t, t[-1] + 1.0), np.append(floors, floors[-1]),
                                              vpr_method="cricavpr", device="cuda")
    msgs = [str(x.message) for x in w]
    assert any("Failed to load image" in m and "zzzz.png" in m for m in msgs)

    ref = mlgate.SemanticPlaceRecognition(vpr_method="cricavpr", device="cuda")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i in sorted(range(n), key=lambda i: f"{t[i]:.6f}.png"):
            img = np.asarray(PIL.open(tmp_path / f"{t[i]:.6f}.png").convert("RGB"))[..., ::-1]
            ref.add_image(image=np.ascontiguousarray(img), timestamp=t[i], floor_label=int(floors[i]),
                          image_path=str(tmp_path / f"{t[i]:.6f}.png"))
        ref_matches = ref.find_loop_closures(enable_floor_gating=True)
    a, b = spr.vpr.descriptors, ref.vpr.descriptors
    assert len(a) == len(b) == n
    for x, y in zip(a, b):
        assert x.timestamp == y.timestamp and x.floor_label == y.floor_label and x.image_path == y.image_path
        # device batch vs one frame per call: same kernels, tiles of another M
        assert np.allclose(x.descriptor, y.descriptor, rtol=0, atol=1e-6)
    assert [(m.query_idx, m.match_idx, m.is_valid) for m in matches] == \
           [(m.query_idx, m.match_idx, m.is_valid) for m in ref_matches]
    assert np.allclose([m.similarity for m in matches], [m.similarity for m in ref_matches], rtol=0, atol=1e-5)
    assert len(matches) > 0 and any(m.is_valid for m in matches)


def test_process_image_sequence_count_mismatch_warns(dev, tmp_path):
    seq = synthetic.make_sequence(4, places=2, seed=5)
    _write(tmp_path, synthetic.frames_host(seq, h=224, w=224), seq.t)
    with pytest.warns(UserWarning, match=r"Number of images \(4\) != timestamps \(3\)"):
        spr, _ = process_image_sequence(tmp_path, seq.t[:3], seq.floor_gt[:3], vpr_method="cricavpr",
                                        device="cuda")
    assert len(spr.vpr.descriptors) == 3
