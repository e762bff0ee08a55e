"""Keyframe ingestion: PNG keyframe files -> BGR uint8 frames in HBM.

Replaces the per-image ``cv2.imread(str(path))`` loop of ``process_image_sequence``
(place_recognition.py:936-991) for the '{timestamp:.6f}.png' keyframes that
``extract_images`` (scripts/utils/bag_utils.py:222-271) writes.  Decoding is host work
(DEFLATE and the PNG row filters are serial per image): ``mlg_png_load_bgr`` decodes a
batch on a pool of host threads straight into a page-locked buffer, and
``KeyframeStream`` copies each batch to HBM on a side stream while the caller's stream
runs the previous batch through the ViT (two pinned buffers, an event per buffer).
"""
import os
import struct
import warnings
import zlib
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import _native

DEFAULT_THREADS = min(16, os.cpu_count() or 1)
_SIG = b"\x89PNG\r\n\x1a\n"


def png_info(data: bytes) -> Optional[Tuple[int, int, int, int]]:
    """(width, height, color_type, bit_depth) from a PNG's IHDR (CRC-checked), None if
    the bytes do not start like a PNG."""
    if len(data) < 33 or data[:8] != _SIG or data[12:16] != b"IHDR" or struct.unpack(">I", data[8:12])[0] != 13:
        return None
    if zlib.crc32(data[12:29]) & 0xFFFFFFFF != struct.unpack(">I", data[29:33])[0]:
        return None
    w, h, depth, ctype = struct.unpack(">IIBB", data[16:26])
    return (w, h, ctype, depth) if w and h else None


def _header(path) -> Optional[Tuple[int, int]]:
    try:
        with open(path, "rb") as f:
            info = png_info(f.read(33))
    except OSError:
        return None
    return None if info is None else (info[1], info[0])


def decode_png_bytes(blobs: Sequence[bytes], H: int, W: int,
                     threads: int = DEFAULT_THREADS) -> Tuple[np.ndarray, np.ndarray]:
    """Decode in-memory PNGs of one size -> (uint8 [n, H, W, 3] BGR, int32 status [n])."""
    import torch
    ts = [torch.frombuffer(bytearray(b), dtype=torch.uint8) if len(b) else torch.zeros(0, dtype=torch.uint8)
          for b in blobs]
    out, status = _native.ops().png_decode(ts, int(H), int(W), int(threads))
    return out.numpy(), status.numpy()


def load_png_batch(paths: Sequence, H: int, W: int, out, threads: int = DEFAULT_THREADS) -> np.ndarray:
    """Decode PNG files of size H x W into the host uint8 tensor ``out`` (>= n*H*W*3
    bytes; page-locked for an async upload); returns the per-file status (0 ok)."""
    return _native.ops().png_load_into([os.fspath(p) for p in paths], out, int(H), int(W), int(threads)).numpy()


def imread(path) -> Optional[np.ndarray]:
    """``cv2.imread(path)`` (IMREAD_COLOR) for a PNG file: BGR uint8 [H, W, 3] or None."""
    import torch
    hw = _header(path)
    if hw is None:
        return None
    out = torch.empty((1, hw[0], hw[1], 3), dtype=torch.uint8)
    st = load_png_batch([path], hw[0], hw[1], out, threads=1)
    return out[0].numpy() if st[0] == 0 else None


def jpeg_reader():
    """A ``path -> BGR uint8 [H, W, 3] or None`` JPEG reader: cv2.imread when OpenCV is
    installed (the reference's call), else Pillow (the same libjpeg-turbo decoder with
    OpenCV's defaults: islow IDCT, fancy upsampling), converted to RGB and channel-swapped.
    Raises the reference's ImportError when neither is available."""
    try:
        import cv2
        return lambda p: cv2.imread(str(p))
    except ImportError:
        pass
    try:
        from PIL import Image
    except ImportError as e:
        raise ImportError("OpenCV is required for image loading. Install with: pip install opencv-python") from e

    def read(p):
        try:
            with Image.open(p) as im:
                return np.ascontiguousarray(np.asarray(im.convert("RGB"))[..., ::-1])
        except (OSError, ValueError):
            return None
    return read


class KeyframeStream:
    """Iterate over PNG keyframes in device batches: yields ``(indices, frames)`` with
    ``frames`` a uint8 [b, H, W, 3] BGR tensor on ``device`` and ``indices`` the positions
    in ``paths`` it holds.  Files that fail to decode are skipped with the reference's
    warning ("Failed to load image: ..."); a file of another size is decoded in a batch
    of its own size.  Decode of batch i + 1 overlaps the caller's work on batch i; the
    upload runs on a side stream and the consumer's stream waits for it by event.
    """

    def __init__(self, paths: Sequence, device="cuda", batch: int = 123, threads: int = DEFAULT_THREADS):
        import torch
        _native.require_device(device)
        self.paths = [str(p) for p in paths]
        self.device = torch.device(device)
        self.batch = int(batch)
        self.threads = int(threads)
        self._torch = torch

    def _groups(self) -> List[Tuple[Tuple[int, int], List[int]]]:
        """Consecutive runs of one frame size, in file order, at most `batch` long."""
        groups, cur, cur_hw = [], [], None
        for i, p in enumerate(self.paths):
            hw = _header(p)
            if hw is None:
                warnings.warn(f"Failed to load image: {p}")
                continue
            if cur and (hw != cur_hw or len(cur) == self.batch):
                groups.append((cur_hw, cur))
                cur = []
            cur_hw = hw
            cur.append(i)
        if cur:
            groups.append((cur_hw, cur))
        return groups

    def __iter__(self) -> Iterator[Tuple[List[int], "object"]]:
        torch = self._torch
        side = torch.cuda.Stream(device=self.device)
        consumer = torch.cuda.current_stream(self.device)
        pinned = [None, None]
        done = [None, None]
        for g, ((H, W), idx) in enumerate(self._groups()):
            slot = g & 1
            need = len(idx) * H * W * 3
            if done[slot] is not None:
                done[slot].synchronize()  # the upload that last read this pinned buffer finished
            if pinned[slot] is None or pinned[slot].numel() < need:
                pinned[slot] = torch.empty(need, dtype=torch.uint8, pin_memory=True)
            host = pinned[slot]
            status = load_png_batch([self.paths[i] for i in idx], H, W, host, self.threads)
            ok = [k for k, s in enumerate(status) if s == 0]
            for k, s in enumerate(status):
                if s != 0:
                    warnings.warn(f"Failed to load image: {self.paths[idx[k]]}")
            if not ok:
                continue
            frames = torch.empty((len(idx), H, W, 3), dtype=torch.uint8, device=self.device)
            side.wait_stream(consumer)  # `frames` may reuse memory the consumer still reads
            with torch.cuda.stream(side):
                frames.copy_(host[:need].view(len(idx), H, W, 3), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
            done[slot] = ev
            consumer.wait_event(ev)
            frames.record_stream(consumer)
            if len(ok) != len(idx):
                frames = frames[torch.tensor(ok, device=self.device)]
            yield [idx[k] for k in ok], frames
        for ev in done:
            if ev is not None:
                ev.synchronize()
