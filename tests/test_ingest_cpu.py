"""Keyframe ingestion: the native PNG loader against lossless round trips.

The loader replaces process_image_sequence's cv2.imread (place_recognition.py:965-968)
of the PNGs bag_utils.extract_images writes (scripts/utils/bag_utils.py:222-271).
OpenCV is not importable here, so parity is pinned two ways: (1) PNG is lossless, so
the decoded BGR frame must equal the array that was encoded -- by Pillow (the
writer's own filter choice) and by the test's own encoder below, which forces each of
the five row filters and Adam7 interlacing; (2) Pillow's decoder (libpng-compatible)
on the same bytes, converted to RGB and channel-swapped, is the IMREAD_COLOR image
for every colour type it covers.  Host-only: no GPU needed.
"""
import io
import struct
import zlib

import numpy as np
import pytest

PIL = pytest.importorskip("PIL.Image")

from mlgate import ingest  # noqa: E402

RNG = np.random.default_rng(7)


def _chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xFFFFFFFF)


def _filter_row(ft, row, prev, bpp):
    out = np.empty_like(row)
    r, p = row.astype(np.int32), prev.astype(np.int32)
    a = np.concatenate([np.zeros(bpp, np.int32), r[:-bpp]])
    c = np.concatenate([np.zeros(bpp, np.int32), p[:-bpp]])
    if ft == 0:
        out = r
    elif ft == 1:
        out = r - a
    elif ft == 2:
        out = r - p
    elif ft == 3:
        out = r - ((a + p) >> 1)
    else:
        pp = a + p - c
        pa, pb, pc = np.abs(pp - a), np.abs(pp - p), np.abs(pp - c)
        pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, p, c))
        out = r - pred
    return (out & 0xFF).astype(np.uint8)


def _raw_rows(img, bpp, filters):
    """Filtered scanlines of a packed byte image [rows, rowbytes]."""
    out = bytearray()
    prev = np.zeros(img.shape[1], np.uint8)
    for y in range(img.shape[0]):
        ft = filters[y % len(filters)]
        out.append(ft)
        out += _filter_row(ft, img[y], prev, bpp).tobytes()
        prev = img[y]
    return bytes(out)


ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def encode_png(pix, ctype, depth=8, filters=(0, 1, 2, 3, 4), interlace=False, plte=None):
    """Minimal PNG writer: pix [H, W, samples] of `depth`-bit samples (8 or 16)."""
    H, W = pix.shape[:2]
    spp = pix.shape[2]
    if depth == 16:
        packed = pix.astype(">u2").view(np.uint8).reshape(H, W, spp * 2)
    else:
        packed = pix.astype(np.uint8)
    bpp = packed.shape[2]

    def rows_of(sub):
        return _raw_rows(sub.reshape(sub.shape[0], -1), bpp, filters)

    if interlace:
        raw = b"".join(rows_of(packed[y0::dy, x0::dx]) for x0, y0, dx, dy in ADAM7
                       if packed[y0::dy, x0::dx].size)
    else:
        raw = rows_of(packed)
    ihdr = struct.pack(">IIBBBBB", W, H, depth, ctype, 0, 0, 1 if interlace else 0)
    body = _chunk(b"IHDR", ihdr)
    if plte is not None:
        body += _chunk(b"PLTE", plte.astype(np.uint8).tobytes())
    # split the stream over several IDAT chunks
    z = zlib.compress(raw, 6)
    for i in range(0, len(z), 4096):
        body += _chunk(b"IDAT", z[i:i + 4096])
    return b"\x89PNG\r\n\x1a\n" + body + _chunk(b"IEND", b"")


def _decode(blob, H, W):
    out, st = ingest.decode_png_bytes([blob], H, W, threads=1)
    return out[0], int(st[0])


def _pil_bgr(blob):
    return np.asarray(PIL.open(io.BytesIO(blob)).convert("RGB"))[..., ::-1]


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("filters", [(0,), (1,), (2,), (3,), (4,), (0, 1, 2, 3, 4)])
def test_rgb8_every_filter(filters, interlace):
    rgb = RNG.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    blob = encode_png(rgb, 2, filters=filters, interlace=interlace)
    bgr, st = _decode(blob, 37, 53)
    assert st == 0
    assert np.array_equal(bgr, rgb[..., ::-1])
    assert np.array_equal(bgr, _pil_bgr(blob))


@pytest.mark.parametrize("mode", ["RGB", "RGBA", "L", "LA", "P", "1"])
def test_pillow_written_modes(mode):
    rgb = RNG.integers(0, 256, (48, 64, 3), dtype=np.uint8)
    im = PIL.fromarray(rgb).convert(mode)
    buf = io.BytesIO()
    im.save(buf, format="PNG")
    blob = buf.getvalue()
    bgr, st = _decode(blob, 48, 64)
    assert st == 0
    assert np.array_equal(bgr, _pil_bgr(blob))


@pytest.mark.parametrize("depth", [1, 2, 4])
def test_low_bit_gray_scaled(depth):
    g = RNG.integers(0, 1 << depth, (9, 21), dtype=np.uint16)
    per = 8 // depth
    W = g.shape[1]
    padded = np.zeros((9, -(-W // per) * per), np.uint16)
    padded[:, :W] = g
    packed = np.zeros((9, padded.shape[1] // per), np.uint8)
    for k in range(per):
        packed |= (padded[:, k::per] << (8 - depth * (k + 1))).astype(np.uint8)
    blob = encode_png(packed[..., None], 0, depth=8, filters=(4,))
    # patch IHDR's bit depth (the writer packs the bytes itself) and the chunk CRC
    ihdr = struct.pack(">IIBBBBB", W, 9, depth, 0, 0, 0, 0)
    blob = blob[:8] + _chunk(b"IHDR", ihdr) + blob[33:]
    bgr, st = _decode(blob, 9, W)
    assert st == 0
    want = (g * (255 // ((1 << depth) - 1))).astype(np.uint8)
    assert np.array_equal(bgr, np.repeat(want[..., None], 3, axis=2))
    assert np.array_equal(bgr, _pil_bgr(blob))


def test_sixteen_bit_high_byte():
    rgb16 = RNG.integers(0, 65536, (11, 13, 3), dtype=np.uint16)
    blob = encode_png(rgb16, 2, depth=16, filters=(0, 4, 3))
    bgr, st = _decode(blob, 11, 13)
    assert st == 0
    assert np.array_equal(bgr, (rgb16 >> 8).astype(np.uint8)[..., ::-1])
    g16 = RNG.integers(0, 65536, (5, 7, 1), dtype=np.uint16)
    bgr, st = _decode(encode_png(g16, 0, depth=16, interlace=True), 5, 7)
    assert st == 0 and np.array_equal(bgr[..., 1], (g16[..., 0] >> 8).astype(np.uint8))


def test_palette_interlaced():
    plte = RNG.integers(0, 256, (16, 3), dtype=np.uint8)
    idx = RNG.integers(0, 16, (19, 23, 1), dtype=np.uint8)
    bgr, st = _decode(encode_png(idx, 3, plte=plte, interlace=True), 19, 23)
    assert st == 0 and np.array_equal(bgr, plte[idx[..., 0]][..., ::-1])


def test_failures_and_sizes(tmp_path):
    rgb = RNG.integers(0, 256, (16, 24, 3), dtype=np.uint8)
    blob = encode_png(rgb, 2)
    assert _decode(blob, 16, 25)[1] == -4                   # MLG_ESIZE
    bad = bytearray(blob)
    bad[40] ^= 0xFF                                         # inside IDAT: CRC mismatch
    assert _decode(bytes(bad), 16, 24)[1] == -1
    assert _decode(blob[:-20], 16, 24)[1] == -1             # truncated
    assert _decode(b"not a png at all" * 4, 16, 24)[1] == -1
    assert ingest.png_info(blob)[:2] == (24, 16)
    p = tmp_path / "1.000000.png"
    p.write_bytes(blob)
    assert np.array_equal(ingest.imread(p), rgb[..., ::-1])
    (tmp_path / "x.png").write_bytes(b"garbage")
    assert ingest.imread(tmp_path / "x.png") is None
    assert ingest.imread(tmp_path / "missing.png") is None


def test_batch_threads_match_single():
    frames = [RNG.integers(0, 256, (30, 40, 3), dtype=np.uint8) for _ in range(12)]
    blobs = [encode_png(f, 2, filters=((i % 5),)) for i, f in enumerate(frames)]
    out, st = ingest.decode_png_bytes(blobs, 30, 40, threads=8)
    assert (st == 0).all()
    for i, f in enumerate(frames):
        assert np.array_equal(out[i], f[..., ::-1])


def test_file_loader(tmp_path):
    frames = [RNG.integers(0, 256, (24, 32, 3), dtype=np.uint8) for _ in range(5)]
    paths = []
    for i, f in enumerate(frames):
        p = tmp_path / f"{i:06d}.png"
        PIL.fromarray(f).save(p)
        paths.append(p)
    import torch
    buf = torch.zeros((5, 24, 32, 3), dtype=torch.uint8)
    st = ingest.load_png_batch(paths, 24, 32, buf, threads=4)
    out = buf.numpy()
    assert (st == 0).all()
    for i, f in enumerate(frames):
        assert np.array_equal(out[i], f[..., ::-1])


def test_jpeg_reader_without_opencv(tmp_path):
    """*.jpg keyframes: cv2.imread when OpenCV exists, else Pillow's libjpeg decode (BGR)."""
    yy, xx = np.mgrid[0:40, 0:56]
    rgb = np.stack([xx * 4, yy * 6, (xx + yy) * 2], -1).astype(np.uint8)  # smooth: JPEG-friendly
    p = tmp_path / "2.000000.jpg"
    PIL.fromarray(rgb).save(p, quality=95)
    read = ingest.jpeg_reader()
    got = read(p)
    assert got.shape == (40, 56, 3) and got.dtype == np.uint8
    assert np.array_equal(got, np.asarray(PIL.open(p).convert("RGB"))[..., ::-1])
    assert np.abs(got.astype(int) - rgb[..., ::-1]).mean() < 8  # lossy, but the same image
    (tmp_path / "bad.jpg").write_bytes(b"\xff\xd8 nope")
    assert read(tmp_path / "bad.jpg") is None
