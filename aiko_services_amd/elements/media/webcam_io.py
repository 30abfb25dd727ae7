"""Webcam source (reference ``elements/media/webcam_io.py``); implementation in video_io."""
from .video_io import VideoReadWebcam  # noqa: F401

__all__ = ["VideoReadWebcam"]
