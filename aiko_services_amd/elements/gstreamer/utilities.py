"""GStreamer helpers (reference ``elements/gstreamer/utilities.py:1-95``)."""
from __future__ import annotations

import sys

__all__ = ["GStreamerError", "enable_opencv", "get_format", "get_h264_decoder", "get_h264_encoder",
           "get_h264_encoder_options", "gst_initialise", "process_video"]

OPERATING_SYSTEM = "mac_os_x" if sys.platform == "darwin" else "linux"
FORMAT = "RGB"
H264_DECODER = {"linux": "avdec_h264", "mac_os_x": "avdec_h264"}
H264_ENCODER = {"linux": "x264enc", "mac_os_x": "vtenc_h264"}

_GST = None


class GStreamerError(Exception):
    def __init__(self, message):
        super().__init__(message)
        self.message = message


def get_format() -> str:
    return FORMAT


def get_h264_decoder() -> str:
    return H264_DECODER[OPERATING_SYSTEM]


def get_h264_encoder() -> str:
    return H264_ENCODER[OPERATING_SYSTEM]


def get_h264_encoder_options() -> str:
    if OPERATING_SYSTEM != "linux":
        return ""
    return "tune=zerolatency speed-preset=ultrafast sliced-threads=true key-int-max=30"


def gst_initialise(multiple_return_values=False):
    """Import and initialise Gst once; GStreamerError when GStreamer is not installed."""
    global _GST
    if _GST is None:
        try:
            import gi
            gi.require_version("Gst", "1.0")
            gi.require_version("GstBase", "1.0")
            from gi.repository import GObject, Gst, GstBase
        except (ImportError, ValueError) as exc:
            raise GStreamerError(f"GStreamer (gi Gst 1.0 typelib) is not available: {exc}") from exc
        Gst.init(None)
        _GST = (Gst, GstBase, GObject)
    return _GST if multiple_return_values else _GST[0]


def enable_opencv():
    try:
        return __import__("cv2")
    except ImportError:
        return None


def process_video(video_reader, video_writer, show=False, limit=None):
    """Copy frames from a reader to a writer until the reader ends (reference helper)."""
    cv2 = enable_opencv() if show else None
    count = 0
    while limit is None or count < limit:
        frame = video_reader.read_frame(0.01)
        if frame is None:
            if getattr(video_reader, "finished", False):
                break
            continue
        if frame.get("type") == "image":
            if cv2 is not None:
                cv2.imshow("Video", cv2.cvtColor(frame["image"], cv2.COLOR_RGB2BGR))
                if cv2.waitKey(1) & 0xFF == ord("q"):
                    break
            video_writer.write_frame(frame)
            count += 1
    return count
