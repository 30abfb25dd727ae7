"""Minimal Video4Linux2 camera capture (no OpenCV): the webcam source of ``webcam_io``.

The reference's ``VideoReadWebcam`` (``/root/reference/src/aiko_services/elements/media/
webcam_io.py``) reads frames through ``cv2.VideoCapture``; OpenCV is not in this image, so the
camera is driven directly through the kernel's V4L2 API: ``VIDIOC_QUERYCAP`` (capture +
streaming capabilities), ``VIDIOC_S_FMT`` (YUYV 4:2:2 at the requested size — the format every
UVC webcam offers), ``VIDIOC_REQBUFS`` / ``VIDIOC_QUERYBUF`` + ``mmap`` (a ring of driver
buffers mapped into the process), ``VIDIOC_QBUF`` / ``VIDIOC_DQBUF`` with ``select`` for
frames, ``VIDIOC_STREAMON`` / ``STREAMOFF``.  Frames are converted YUYV -> RGB (BT.601, studio
range) with numpy.  Struct layouts and ioctl numbers are those of ``linux/videodev2.h`` on
64-bit Linux.
"""
from __future__ import annotations

import ctypes
import errno
import fcntl
import mmap
import os
import select

import numpy as np

__all__ = ["V4L2Capture", "yuyv_to_rgb", "VIDIOC", "fourcc"]

_IOC_WRITE, _IOC_READ = 1, 2


def _ioc(direction, nr, size, kind=ord("V")):
    return (direction << 30) | (size << 16) | (kind << 8) | nr


def fourcc(code: str) -> int:
    a, b, c, d = (ord(ch) for ch in code)
    return a | (b << 8) | (c << 16) | (d << 24)


class v4l2_capability(ctypes.Structure):
    _fields_ = [("driver", ctypes.c_char * 16), ("card", ctypes.c_char * 32), ("bus_info", ctypes.c_char * 32),
                ("version", ctypes.c_uint32), ("capabilities", ctypes.c_uint32),
                ("device_caps", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 3)]


class v4l2_pix_format(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("pixelformat", ctypes.c_uint32),
                ("field", ctypes.c_uint32), ("bytesperline", ctypes.c_uint32), ("sizeimage", ctypes.c_uint32),
                ("colorspace", ctypes.c_uint32), ("priv", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("ycbcr_enc", ctypes.c_uint32), ("quantization", ctypes.c_uint32), ("xfer_func", ctypes.c_uint32)]


class _fmt_union(ctypes.Union):
    _fields_ = [("pix", v4l2_pix_format), ("raw_data", ctypes.c_uint8 * 200), ("_align", ctypes.c_uint64)]


class v4l2_format(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint32), ("fmt", _fmt_union)]


class v4l2_requestbuffers(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint32), ("type", ctypes.c_uint32), ("memory", ctypes.c_uint32),
                ("capabilities", ctypes.c_uint32), ("flags", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3)]


class timeval(ctypes.Structure):
    _fields_ = [("tv_sec", ctypes.c_long), ("tv_usec", ctypes.c_long)]


class v4l2_timecode(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("frames", ctypes.c_uint8),
                ("seconds", ctypes.c_uint8), ("minutes", ctypes.c_uint8), ("hours", ctypes.c_uint8),
                ("userbits", ctypes.c_uint8 * 4)]


class _buf_m(ctypes.Union):
    _fields_ = [("offset", ctypes.c_uint32), ("userptr", ctypes.c_ulong), ("planes", ctypes.c_void_p),
                ("fd", ctypes.c_int32)]


class v4l2_buffer(ctypes.Structure):
    _fields_ = [("index", ctypes.c_uint32), ("type", ctypes.c_uint32), ("bytesused", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("field", ctypes.c_uint32), ("timestamp", timeval),
                ("timecode", v4l2_timecode), ("sequence", ctypes.c_uint32), ("memory", ctypes.c_uint32),
                ("m", _buf_m), ("length", ctypes.c_uint32), ("reserved2", ctypes.c_uint32),
                ("request_fd", ctypes.c_int32)]


BUF_TYPE_VIDEO_CAPTURE = 1
MEMORY_MMAP = 1
FIELD_ANY = 0
CAP_VIDEO_CAPTURE = 0x00000001
CAP_STREAMING = 0x04000000
PIX_FMT_YUYV = fourcc("YUYV")

VIDIOC = {
    "QUERYCAP": _ioc(_IOC_READ, 0, ctypes.sizeof(v4l2_capability)),
    "S_FMT": _ioc(_IOC_READ | _IOC_WRITE, 5, ctypes.sizeof(v4l2_format)),
    "REQBUFS": _ioc(_IOC_READ | _IOC_WRITE, 8, ctypes.sizeof(v4l2_requestbuffers)),
    "QUERYBUF": _ioc(_IOC_READ | _IOC_WRITE, 9, ctypes.sizeof(v4l2_buffer)),
    "QBUF": _ioc(_IOC_READ | _IOC_WRITE, 15, ctypes.sizeof(v4l2_buffer)),
    "DQBUF": _ioc(_IOC_READ | _IOC_WRITE, 17, ctypes.sizeof(v4l2_buffer)),
    "STREAMON": _ioc(_IOC_WRITE, 18, ctypes.sizeof(ctypes.c_int)),
    "STREAMOFF": _ioc(_IOC_WRITE, 19, ctypes.sizeof(ctypes.c_int)),
}


def yuyv_to_rgb(buf, width: int, height: int) -> np.ndarray:
    """Packed YUYV 4:2:2 (Y0 U Y1 V per pixel pair) -> uint8 RGB [H, W, 3], BT.601 studio range."""
    a = np.frombuffer(buf, dtype=np.uint8, count=width * height * 2).reshape(height, width // 2, 4)
    a = a.astype(np.float32)
    y = np.empty((height, width), np.float32)
    y[:, 0::2], y[:, 1::2] = a[..., 0], a[..., 2]
    u = np.repeat(a[..., 1], 2, axis=1) - 128.0
    v = np.repeat(a[..., 3], 2, axis=1) - 128.0
    c = (y - 16.0) * 1.164383
    rgb = np.stack([c + 1.596027 * v, c - 0.391762 * u - 0.812968 * v, c + 2.017232 * u], axis=-1)
    return np.clip(np.rint(rgb), 0, 255).astype(np.uint8)


class V4L2Capture:
    """``cv2.VideoCapture``-like camera reader: ``isOpened()``, ``read() -> (ok, rgb)``,
    ``release()``.  ``path``: ``/dev/videoN`` or an integer N."""

    def __init__(self, path="/dev/video0", width: int = 640, height: int = 480, buffers: int = 4,
                 timeout_s: float = 2.0):
        if isinstance(path, int) or (isinstance(path, str) and path.isdigit()):
            path = f"/dev/video{int(path)}"
        self.path, self.timeout_s = path, timeout_s
        self.fd = os.open(path, os.O_RDWR | os.O_NONBLOCK)
        self.maps = []
        self.streaming = False
        try:
            cap = v4l2_capability()
            fcntl.ioctl(self.fd, VIDIOC["QUERYCAP"], cap)
            caps = cap.device_caps or cap.capabilities
            if not caps & CAP_VIDEO_CAPTURE or not caps & CAP_STREAMING:
                raise OSError(errno.ENODEV, f"{path}: not a streaming video capture device")
            fmt = v4l2_format()
            fmt.type = BUF_TYPE_VIDEO_CAPTURE
            fmt.fmt.pix.width, fmt.fmt.pix.height = width, height
            fmt.fmt.pix.pixelformat, fmt.fmt.pix.field = PIX_FMT_YUYV, FIELD_ANY
            fcntl.ioctl(self.fd, VIDIOC["S_FMT"], fmt)
            if fmt.fmt.pix.pixelformat != PIX_FMT_YUYV:
                raise OSError(errno.EINVAL, f"{path}: YUYV capture not supported")
            self.width, self.height = fmt.fmt.pix.width, fmt.fmt.pix.height
            req = v4l2_requestbuffers(count=buffers, type=BUF_TYPE_VIDEO_CAPTURE, memory=MEMORY_MMAP)
            fcntl.ioctl(self.fd, VIDIOC["REQBUFS"], req)
            for i in range(req.count):
                b = v4l2_buffer(index=i, type=BUF_TYPE_VIDEO_CAPTURE, memory=MEMORY_MMAP)
                fcntl.ioctl(self.fd, VIDIOC["QUERYBUF"], b)
                self.maps.append(mmap.mmap(self.fd, b.length, mmap.MAP_SHARED,
                                           mmap.PROT_READ | mmap.PROT_WRITE, offset=b.m.offset))
                fcntl.ioctl(self.fd, VIDIOC["QBUF"], b)
            fcntl.ioctl(self.fd, VIDIOC["STREAMON"], ctypes.c_int(BUF_TYPE_VIDEO_CAPTURE))
            self.streaming = True
        except BaseException:
            self.release()
            raise

    def isOpened(self) -> bool:  # noqa: N802  (cv2.VideoCapture API)
        return self.fd is not None and self.streaming

    def read(self):
        """(True, RGB uint8 [H, W, 3]) for the next frame, (False, None) on timeout / error."""
        if not self.isOpened():
            return False, None
        ready, _, _ = select.select([self.fd], [], [], self.timeout_s)
        if not ready:
            return False, None
        b = v4l2_buffer(type=BUF_TYPE_VIDEO_CAPTURE, memory=MEMORY_MMAP)
        try:
            fcntl.ioctl(self.fd, VIDIOC["DQBUF"], b)
        except OSError:
            return False, None
        try:
            rgb = yuyv_to_rgb(self.maps[b.index][:b.bytesused], self.width, self.height)
        finally:
            fcntl.ioctl(self.fd, VIDIOC["QBUF"], b)
        return True, rgb

    def release(self):
        if self.fd is None:
            return
        if self.streaming:
            try:
                fcntl.ioctl(self.fd, VIDIOC["STREAMOFF"], ctypes.c_int(BUF_TYPE_VIDEO_CAPTURE))
            except OSError:
                pass
            self.streaming = False
        for m in self.maps:
            m.close()
        self.maps = []
        os.close(self.fd)
        self.fd = None
