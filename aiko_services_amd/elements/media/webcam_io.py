"""Webcam source (reference ``elements/media/webcam_io.py:61-144``).

``VideoReadWebcam`` generates a frame per camera image with the reference's EC-tunable share
items: ``color`` (RGB or grey), ``flip`` (none / horizontal / vertical / both), ``path`` (the
device; changing it re-opens the camera) and ``frame_id`` (published every 10 frames).  The
camera is read through OpenCV when it is installed, otherwise directly through Video4Linux2
(``v4l2.py``: mmap'd YUYV buffers, converted to RGB in numpy) — this image has no OpenCV, so the
V4L2 path is the one that runs here.  Parameters ``width`` / ``height`` (default 640 x 480)
request the capture size.
"""
from __future__ import annotations

import numpy as np

from ...pipeline.stream import StreamEvent
from .common_io import DataSource

try:  # optional
    import cv2  # type: ignore
    _CV2 = True
except ImportError:
    cv2 = None
    _CV2 = False

__all__ = ["VideoReadWebcam", "open_camera", "postprocess_frame"]


def open_camera(path, width: int = 640, height: int = 480):
    """A ``cv2.VideoCapture``-like reader for ``path`` (``/dev/videoN`` or N) whose ``read()``
    returns RGB frames; OpenCV when available (its BGR converted), else V4L2."""
    if _CV2:
        cap = cv2.VideoCapture(path)
        if not cap.isOpened():
            raise OSError(f"cannot open camera {path}")

        class _RGB:
            def isOpened(self):  # noqa: N802
                return cap.isOpened()

            def read(self):
                ok, bgr = cap.read()
                return ok, (cv2.cvtColor(bgr, cv2.COLOR_BGR2RGB) if ok else None)

            def release(self):
                cap.release()
        return _RGB()
    from .v4l2 import V4L2Capture
    return V4L2Capture(path, width, height)


def postprocess_frame(rgb: np.ndarray, color=True, flip="none") -> np.ndarray:
    """The share's ``color`` (False: BT.601 luma) / ``flip`` settings applied to one RGB frame."""
    image = rgb
    if not color:
        image = np.rint(rgb.astype(np.float32) @ np.array([0.299, 0.587, 0.114], np.float32))
        image = np.clip(image, 0, 255).astype(np.uint8)
    if flip in ("both", "horizontal"):
        image = image[:, ::-1]
    if flip in ("both", "vertical"):
        image = image[::-1]
    return np.ascontiguousarray(image)


class VideoReadWebcam(DataSource):
    """Camera source with EC-tunable ``color``, ``flip``, ``path``."""

    def __init__(self, context):
        context.set_protocol("webcam:0")
        context.get_implementation("PipelineElement").__init__(self, context)
        self.path_current = None
        self.stream_started = 0
        self.video_capture = None
        self.share["color"] = True
        self.share["flip"] = "none"
        self.share["frame_id"] = -1
        self.share["path"] = "/dev/video0"
        self.ec_producer.add_handler(self._ec_producer_change_handler)

    def _ec_producer_change_handler(self, command, item_name, item_value):
        if item_name == "color" and isinstance(item_value, str):
            self.share["color"] = item_value.lower() == "true"
        if item_name == "path":
            if isinstance(item_value, str) and item_value.isdigit():
                item_value = int(item_value)
            if item_value != self.path_current and self.stream_started:
                self._open_camera(item_value)

    def _open_camera(self, path) -> bool:
        if self.video_capture is not None:
            self.video_capture.release()
            self.video_capture = None
        width = int(self.get_parameter("width", 640)[0])
        height = int(self.get_parameter("height", 480)[0])
        try:
            self.video_capture = open_camera(path, width, height)
        except OSError as exc:
            self.logger.error(f"Open camera: {path} failed: {exc}")
            return False
        self.path_current = path
        self.share["path"] = path
        return True

    def start_stream(self, stream, stream_id):
        self.stream_started += 1
        path, _ = self.get_parameter("path", "/dev/video0")
        if not self._open_camera(path):
            self.stream_started -= 1
            return StreamEvent.ERROR, {"diagnostic": f"VideoReadWebcam: cannot open camera {path}"}
        self.create_frames(stream, self.frame_generator, rate=None)
        return StreamEvent.OKAY, {}

    def frame_generator(self, stream, frame_id):
        if self.video_capture is None or not self.video_capture.isOpened():
            return StreamEvent.DROP_FRAME, {}
        ok, rgb = self.video_capture.read()
        if not ok:
            return StreamEvent.DROP_FRAME, {}
        if frame_id % 10 == 0:
            self.ec_producer.update("frame_id", frame_id)
        return StreamEvent.OKAY, {"images": [self.postprocess(rgb)]}

    def postprocess(self, rgb: np.ndarray) -> np.ndarray:
        return postprocess_frame(rgb, self.share["color"], self.share["flip"])

    def process_frame(self, stream, images):
        return StreamEvent.OKAY, {"images": images}

    def stop_stream(self, stream, stream_id):
        self.stream_started = max(0, self.stream_started - 1)
        if self.stream_started == 0 and self.video_capture is not None:
            self.video_capture.release()
            self.video_capture = None
        return StreamEvent.OKAY, {}
