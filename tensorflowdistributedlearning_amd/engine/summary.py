"""Summaries: JSONL log + TensorBoard-compatible event files, written by rank 0.

The reference writes TF summaries via ``SummarySaverHook`` every 20 train steps to
``fold{i}/train`` and every eval step to ``fold{i}/eval`` (model.py:470-481; scalars
``metrics/mean_acc``, ``metrics/mean_iou``, ``loss/lovasz_loss``).  TensorBoard is not
installed here, so the event format is produced directly: TFRecord framing (length, masked
CRC32C of length, payload, masked CRC32C of payload) around hand-encoded ``Event`` protobufs
(wall_time=1:double, step=2:int64, summary=5:Summary{value=1:Value{tag=1:string,
simple_value=2:float | image=4:Image{height=1, width=2, colorspace=3,
encoded_image_string=4}}}).  Files are readable by TensorBoard's event loader.  Image summaries
(the reference's ``tf.summary.image`` of input/label/probability/prediction, model.py:405-440)
are PNG-encoded here with zlib.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import threading
import time
import zlib

# ----------------------------------------------------------------------------------------------
# CRC32C (Castagnoli), table driven
# ----------------------------------------------------------------------------------------------
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def _native_crc():
    try:
        from .. import _native
        return _native.load().crc32c
    except Exception:  # noqa: BLE001 — no extension: the Python table loop below
        return None


_NATIVE_CRC = [None, False]


def crc32c(data: bytes) -> int:
    if not _NATIVE_CRC[1]:
        _NATIVE_CRC[0], _NATIVE_CRC[1] = _native_crc(), True
    if _NATIVE_CRC[0] is not None:
        return _NATIVE_CRC[0](bytes(data))
    return crc32c_py(data)


def crc32c_py(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc = _TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ----------------------------------------------------------------------------------------------
# minimal protobuf encoding
# ----------------------------------------------------------------------------------------------
def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wire):
    return _varint((field << 3) | wire)


def _len_delim(field, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_scalar_event(tag: str, value: float, step: int, wall_time: float) -> bytes:
    v = _len_delim(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(value))
    summary = _len_delim(1, v)
    ev = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    ev += _len_delim(5, summary)
    return ev


def encode_png_gray(img) -> bytes:
    """[H, W] or [H, W, 1] array in [0, 1] → 8-bit grayscale PNG bytes."""
    import numpy as np
    a = np.asarray(img, dtype=np.float32)
    if a.ndim == 3:
        a = a[..., 0]
    a = (np.clip(a, 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)
    h, w = a.shape
    raw = b"".join(b"\x00" + a[i].tobytes() for i in range(h))

    def chunk(kind, data):
        c = kind + data
        return struct.pack(">I", len(data)) + c + struct.pack(">I", zlib.crc32(c) & 0xFFFFFFFF)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(raw, 6))
            + chunk(b"IEND", b""))


def encode_image_event(tag: str, png: bytes, h: int, w: int, step: int, wall_time: float) -> bytes:
    im = _key(1, 0) + _varint(h) + _key(2, 0) + _varint(w) + _key(3, 0) + _varint(1)
    im += _len_delim(4, png)
    v = _len_delim(1, tag.encode()) + _len_delim(4, im)
    ev = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    ev += _len_delim(5, _len_delim(1, v))
    return ev


def encode_file_version_event(wall_time: float) -> bytes:
    return _key(1, 1) + struct.pack("<d", wall_time) + _len_delim(3, b"brain.Event:2")


def tfrecord(payload: bytes) -> bytes:
    hdr = struct.pack("<Q", len(payload))
    return hdr + struct.pack("<I", _masked_crc(hdr)) + payload + struct.pack("<I", _masked_crc(payload))


def read_tfrecords(path):
    """Iterate payloads of a TFRecord file, verifying CRCs (used by tests)."""
    with open(path, "rb") as f:
        data = f.read()
    off = 0
    while off < len(data):
        (n,) = struct.unpack_from("<Q", data, off)
        (hc,) = struct.unpack_from("<I", data, off + 8)
        assert hc == _masked_crc(data[off:off + 8]), "header crc"
        payload = data[off + 12: off + 12 + n]
        (pc,) = struct.unpack_from("<I", data, off + 12 + n)
        assert pc == _masked_crc(payload), "payload crc"
        yield payload
        off += 16 + n


class SummaryWriter:
    """Scalar summaries to ``<logdir>/events.out.tfevents.*`` and ``<logdir>/scalars.jsonl``."""

    def __init__(self, logdir, enabled=True):
        self.enabled = enabled
        self.logdir = logdir
        self._ev = None
        self._js = None
        self._lock = threading.Lock()  # event-file writes from the caller and the image worker
        self._pool = None
        if enabled:
            os.makedirs(logdir, exist_ok=True)
            now = time.time()
            fname = f"events.out.tfevents.{int(now)}.{socket.gethostname()}"
            self._ev = open(os.path.join(logdir, fname), "ab")
            self._ev.write(tfrecord(encode_file_version_event(now)))
            self._js = open(os.path.join(logdir, "scalars.jsonl"), "a")

    def scalar(self, tag, value, step):
        if not self.enabled:
            return
        now = time.time()
        rec = tfrecord(encode_scalar_event(tag, float(value), int(step), now))
        with self._lock:
            self._ev.write(rec)
            self._js.write(json.dumps({"step": int(step), "tag": tag, "value": float(value),
                                       "wall_time": now}) + "\n")

    def image(self, tag, img, step):
        """Grayscale image summary; ``img`` [H, W(, 1)] with values in [0, 1]."""
        if not self.enabled:
            return
        import numpy as np
        a = np.asarray(img, dtype=np.float32)
        h, w = a.shape[:2]
        rec = tfrecord(encode_image_event(tag, encode_png_gray(a), h, w, int(step), time.time()))
        with self._lock:
            self._ev.write(rec)

    def images_async(self, items, step):
        """``[(tag, img), …]`` PNG-encoded and written on a background thread (the training
        thread only hands over host arrays; :meth:`flush` / :meth:`close` wait for it)."""
        if not self.enabled:
            return
        if self._pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(1, thread_name_prefix="tdl-summary")
        self._pool.submit(lambda: [self.image(t, im, step) for t, im in items])

    def _drain(self):
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None

    def scalars(self, d, step):
        for k, v in d.items():
            self.scalar(k, v, step)

    def flush(self):
        if self.enabled:
            self._drain()
            self._ev.flush()
            self._js.flush()

    def close(self):
        if self.enabled:
            self._drain()
            self._ev.close()
            self._js.close()
            self.enabled = False
