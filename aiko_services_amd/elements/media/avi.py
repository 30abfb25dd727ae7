"""AVI (RIFF) video container: Motion-JPEG and uncompressed frames, without OpenCV.

The reference reads and writes video through ``cv2.VideoCapture`` / ``cv2.VideoWriter``
(``/root/reference/src/aiko_services/elements/media/video_io.py``).  OpenCV is not in this
image, so this module handles the container that cameras and ``cv2.VideoWriter`` (fourcc
``MJPG``) most often produce.  Frames are JPEG-coded through Pillow, or stored as uncompressed
bottom-up BGR DIBs.

Layout written (readers accept any chunk order, ``LIST 'rec '`` groups and OpenDML ``AVIX``
continuation RIFFs):

    RIFF 'AVI '
      LIST 'hdrl'  avih (MainAVIHeader)  LIST 'strl' [strh (AVIStreamHeader 'vids'),
                                                      strf (BITMAPINFOHEADER)]
      LIST 'movi'  00dc | 00db chunks (even-padded)
      idx1         (ckid, AVIIF_KEYFRAME, offset from the 'movi' fourcc, size) per frame

Header and index totals (frame count, sizes) are patched when the writer closes.
"""
from __future__ import annotations

import io
import struct
from pathlib import Path

import numpy as np

__all__ = ["AviWriter", "iter_avi", "read_avi", "avi_info", "write_avi"]

_AVIF_HASINDEX = 0x10
_AVIIF_KEYFRAME = 0x10
_BI_RGB = 0


def _pad(n: int) -> int:
    return n + (n & 1)


# ---- reading ---------------------------------------------------------------------------------

def _chunks(f, start: int, end: int):
    """(fourcc, data offset, size, list type or None) of the chunks in [start, end)."""
    pos = start
    while pos + 8 <= end:
        f.seek(pos)
        hdr = f.read(8)
        if len(hdr) < 8:
            return
        cid, size = hdr[:4], struct.unpack("<I", hdr[4:])[0]
        if cid in (b"RIFF", b"LIST"):
            kind = f.read(4)
            yield cid, pos + 12, size - 4, kind
        else:
            yield cid, pos + 8, size, None
        pos += 8 + _pad(size)


def _parse(path):
    """Stream format + the ordered (offset, size, fourcc) of the first video stream's chunks."""
    info, frames = {}, []
    with open(path, "rb") as f:
        f.seek(0, 2)
        file_end = f.tell()
        pos = 0
        riff_seen = False
        while pos + 12 <= file_end:                 # RIFF 'AVI ' then OpenDML RIFF 'AVIX' ...
            f.seek(pos)
            hdr = f.read(12)
            if hdr[:4] != b"RIFF" or hdr[8:12] not in (b"AVI ", b"AVIX"):
                if not riff_seen:
                    raise ValueError(f"{path}: not an AVI file")
                break
            riff_seen = True
            size = struct.unpack("<I", hdr[4:8])[0]
            _walk(f, pos + 12, min(file_end, pos + 8 + size), info, frames)
            pos += 8 + _pad(size)
    if "width" not in info:
        raise ValueError(f"{path}: no video stream header")
    for k in ("_cur", "_nstrl"):
        info.pop(k, None)
    return info, frames


def _walk(f, start, end, info, frames):
    for cid, off, size, kind in _chunks(f, start, end):
        if cid == b"LIST":
            if kind == b"strl":                     # stream headers, numbered in file order
                info["_cur"] = info.get("_nstrl", 0)
                info["_nstrl"] = info["_cur"] + 1
                _walk(f, off, off + size, info, frames)
            elif kind in (b"hdrl", b"movi", b"rec "):
                _walk(f, off, off + size, info, frames)
        elif cid == b"avih":
            f.seek(off)
            us, = struct.unpack("<I", f.read(4))
            info.setdefault("fps", 1e6 / us if us else 0.0)
        elif cid == b"strh":
            f.seek(off)
            d = f.read(min(size, 56))
            if d[:4] == b"vids" and "handler" not in info:
                info["handler"] = d[4:8]
                info["stream"] = b"%02d" % info.get("_cur", 0)
                scale, rate = struct.unpack("<II", d[20:28])
                if scale:
                    info["fps"] = rate / scale
        elif cid == b"strf" and "width" not in info and "handler" in info and info.get("_cur") == int(info["stream"]):
            f.seek(off)
            d = f.read(40)
            (_, w, h, _, bits, comp) = struct.unpack("<IiiHHI", d[:20])
            info.update(width=w, height=abs(h), bottom_up=h > 0, bits=bits,
                        compression=struct.pack("<I", comp))
        elif cid[2:] in (b"dc", b"db") and cid[:2] == info.get("stream", b"00"):
            frames.append((off, size, cid))


def avi_info(path) -> dict:
    """width, height, fps, compression fourcc, frame count of an AVI's first video stream."""
    info, frames = _parse(path)
    return dict(info, frames=len(frames))


def _decode(buf: bytes, cid: bytes, info: dict) -> np.ndarray:
    comp = info["compression"]
    if comp == b"\0\0\0\0" or cid[2:] == b"db":
        w, h, bits = info["width"], info["height"], info["bits"]
        if bits not in (24, 32):
            raise ValueError(f"uncompressed AVI with {bits} bits per pixel is not supported")
        bpp = bits // 8
        stride = (w * bpp + 3) & ~3
        a = np.frombuffer(buf, np.uint8, count=stride * h).reshape(h, stride)[:, :w * bpp]
        a = a.reshape(h, w, bpp)[:, :, 2::-1]       # BGR(A) -> RGB
        if info["bottom_up"]:
            a = a[::-1]
        return np.ascontiguousarray(a)
    if comp.upper() in (b"MJPG", b"JPEG", b"AVRN", b"LJPG", b"DMB1"):
        from PIL import Image
        return np.asarray(Image.open(io.BytesIO(buf)).convert("RGB"))
    raise ValueError(f"AVI codec {comp!r} needs OpenCV (supported here: MJPG, uncompressed)")


def iter_avi(path):
    """RGB uint8 frames [H, W, 3] of an AVI file's first video stream."""
    info, frames = _parse(path)
    with open(path, "rb") as f:
        for off, size, cid in frames:
            if size == 0:                           # dropped-frame marker: repeat nothing
                continue
            f.seek(off)
            yield _decode(f.read(size), cid, info)


def read_avi(path) -> np.ndarray:
    return np.stack(list(iter_avi(path)))


# ---- writing ---------------------------------------------------------------------------------

class AviWriter:
    """``write(rgb)`` frames of one size into ``path``; ``codec`` ``"MJPG"`` (JPEG ``quality``)
    or ``"raw"`` (uncompressed 24-bit DIB, lossless)."""

    def __init__(self, path, width: int, height: int, fps: float = 30.0, codec: str = "MJPG",
                 quality: int = 90):
        if codec not in ("MJPG", "raw"):
            raise ValueError(f"codec must be 'MJPG' or 'raw' (got {codec!r})")
        self.path, self.w, self.h, self.fps = Path(path), int(width), int(height), float(fps)
        self.codec, self.quality = codec, int(quality)
        self.f = open(self.path, "wb")
        self.index = []                             # (ckid, offset from movi fourcc, size)
        self.max_chunk = 0
        self._write_headers()

    def _write_headers(self):
        f = self.f
        us = int(round(1e6 / self.fps)) if self.fps > 0 else 0
        rate, scale = (int(round(self.fps * 1000)), 1000) if self.fps > 0 else (0, 1)
        raw = self.codec == "raw"
        handler = b"DIB " if raw else b"MJPG"
        comp = struct.pack("<I", _BI_RGB) if raw else b"MJPG"
        image_size = ((self.w * 3 + 3) & ~3) * self.h if raw else self.w * self.h * 3
        avih = struct.pack("<14I", us, 0, 0, _AVIF_HASINDEX, 0, 0, 1, 0, self.w, self.h, 0, 0, 0, 0)
        strh = struct.pack("<4s4sIHHIIIIIIIIhhhh", b"vids", handler, 0, 0, 0, 0, scale, rate, 0, 0,
                           0, 0xFFFFFFFF, 0, 0, 0, self.w, self.h)
        strf = struct.pack("<IiiHH4sIiiII", 40, self.w, self.h, 1, 24, comp, image_size, 0, 0, 0, 0)
        strl = b"strl" + b"strh" + struct.pack("<I", len(strh)) + strh + b"strf" + struct.pack("<I", len(strf)) + strf
        hdrl = b"hdrl" + b"avih" + struct.pack("<I", len(avih)) + avih + b"LIST" + struct.pack("<I", len(strl)) + strl
        f.write(b"RIFF\0\0\0\0AVI ")
        self._avih_at = 12 + 8 + 4 + 8                 # RIFF hdr, LIST hdr, 'hdrl', avih hdr
        self._strh_at = self._avih_at + len(avih) + 8 + 4 + 8
        f.write(b"LIST" + struct.pack("<I", len(hdrl)) + hdrl)
        self._movi_at = f.tell()                       # position of 'LIST' of movi
        f.write(b"LIST\0\0\0\0movi")

    def _encode(self, rgb: np.ndarray) -> tuple:
        if self.codec == "raw":
            stride = (self.w * 3 + 3) & ~3
            out = np.zeros((self.h, stride), np.uint8)
            out[:, :self.w * 3] = rgb[::-1, :, ::-1].reshape(self.h, self.w * 3)   # bottom-up BGR
            return b"00db", out.tobytes()
        from PIL import Image
        buf = io.BytesIO()
        Image.fromarray(rgb, "RGB").save(buf, format="JPEG", quality=self.quality)
        return b"00dc", buf.getvalue()

    def write(self, rgb):
        a = np.asarray(rgb)
        if a.ndim == 2:
            a = np.repeat(a[..., None], 3, axis=2)
        if a.shape[:2] != (self.h, self.w) or a.shape[2] != 3:
            raise ValueError(f"frame {a.shape} does not match the video's {self.h}x{self.w}x3")
        cid, data = self._encode(np.ascontiguousarray(a.astype(np.uint8, copy=False)))
        off = self.f.tell() - (self._movi_at + 8)        # from the 'movi' fourcc
        self.f.write(cid + struct.pack("<I", len(data)) + data + (b"\0" if len(data) & 1 else b""))
        self.index.append((cid, off, len(data)))
        self.max_chunk = max(self.max_chunk, len(data))

    def close(self):
        if self.f is None:
            return
        f = self.f
        movi_end = f.tell()
        idx = b"".join(struct.pack("<4sIII", cid, _AVIIF_KEYFRAME, off, size) for cid, off, size in self.index)
        f.write(b"idx1" + struct.pack("<I", len(idx)) + idx)
        end = f.tell()
        n = len(self.index)
        f.seek(4)
        f.write(struct.pack("<I", end - 8))                                   # RIFF size
        f.seek(self._movi_at + 4)
        f.write(struct.pack("<I", movi_end - self._movi_at - 8))              # movi LIST size
        f.seek(self._avih_at + 16)
        f.write(struct.pack("<I", n))                                         # dwTotalFrames
        f.seek(self._avih_at + 28)
        f.write(struct.pack("<I", self.max_chunk))                            # dwSuggestedBufferSize
        f.seek(self._strh_at + 32)
        f.write(struct.pack("<II", n, self.max_chunk))                        # dwLength, buffer size
        f.close()
        self.f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_avi(path, frames, fps: float = 30.0, codec: str = "MJPG", quality: int = 90):
    frames = list(frames)
    h, w = np.asarray(frames[0]).shape[:2]
    with AviWriter(path, w, h, fps, codec, quality) as wr:
        for fr in frames:
            wr.write(fr)
