"""V4L2 webcam backend (no OpenCV in this image): ioctl numbers and struct layouts against
linux/videodev2.h (64-bit), YUYV -> RGB conversion against the BT.601 formula, and the webcam
element's colour / flip post-processing.  No camera is attached here: opening a missing device
must fail with a clear error (the element then ends the stream with a diagnostic)."""
import ctypes

import numpy as np
import pytest

from aiko_services_amd.elements.media import v4l2 as V


def test_ioctl_numbers_and_struct_sizes():
    assert ctypes.sizeof(V.v4l2_capability) == 104
    assert ctypes.sizeof(V.v4l2_format) == 208
    assert ctypes.sizeof(V.v4l2_requestbuffers) == 20
    assert ctypes.sizeof(V.v4l2_buffer) == 88
    assert V.v4l2_buffer.m.offset == 64 and V.v4l2_buffer.length.offset == 72
    assert V.VIDIOC == {"QUERYCAP": 0x80685600, "S_FMT": 0xC0D05605, "REQBUFS": 0xC0145608,
                        "QUERYBUF": 0xC0585609, "QBUF": 0xC058560F, "DQBUF": 0xC0585611,
                        "STREAMON": 0x40045612, "STREAMOFF": 0x40045613}
    assert V.PIX_FMT_YUYV == 0x56595559


def test_yuyv_to_rgb_matches_bt601():
    rng = np.random.default_rng(0)
    W, H = 8, 3
    raw = rng.integers(0, 256, size=(H, W // 2, 4), dtype=np.uint8)
    rgb = V.yuyv_to_rgb(raw.tobytes(), W, H)
    assert rgb.shape == (H, W, 3) and rgb.dtype == np.uint8
    for yy in range(H):
        for x in range(W):
            y0, u, y1, v = raw[yy, x // 2].astype(float)
            y = y0 if x % 2 == 0 else y1
            c = 1.164383 * (y - 16)
            ref = [c + 1.596027 * (v - 128), c - 0.391762 * (u - 128) - 0.812968 * (v - 128), c + 2.017232 * (u - 128)]
            assert np.all(np.abs(rgb[yy, x].astype(float) - np.clip(np.rint(ref), 0, 255)) <= 1)


def test_missing_device_fails_clearly(tmp_path):
    with pytest.raises(OSError):
        V.V4L2Capture(str(tmp_path / "video9"))


def test_webcam_postprocess_colour_and_flip():
    from aiko_services_amd.elements.media.webcam_io import postprocess_frame
    img = np.arange(2 * 3 * 3, dtype=np.uint8).reshape(2, 3, 3)
    assert np.array_equal(postprocess_frame(img, True, "horizontal"), img[:, ::-1])
    grey = postprocess_frame(img, False, "both")
    assert grey.shape == (2, 3) and grey[0, 0] == int(np.rint(img[1, 2] @ [0.299, 0.587, 0.114]))
