"""Video elements (reference ``elements/media/video_io.py:96-308``, ``webcam_io.py:61-144``).

OpenCV is optional (absent on the MI355X boxes).  Without it, video files are read/written
with in-repo codecs: ``.avi`` (RIFF container, Motion-JPEG through Pillow or uncompressed DIB
frames — ``avi.py``; what cameras and ``cv2.VideoWriter('MJPG')`` produce), animated ``.gif``
(Pillow), raw ``.y4m`` (YUV4MPEG2, 4:2:0 / 4:4:4, converted to RGB with BT.601), ``.npy``
arrays ``[T, H, W, 3]`` uint8, and directories of images.  With OpenCV present any other
container it supports works too.
``VideoShow`` needs a display: without one it logs frame statistics instead.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

from ...pipeline.engine import PipelineElement
from ...pipeline.stream import StreamEvent
from .avi import AviWriter, iter_avi
from .common_io import DataSource, DataTarget, contains_all

try:  # optional
    import cv2  # type: ignore
    _CV2 = True
except ImportError:
    cv2 = None
    _CV2 = False

__all__ = ["VideoOutput", "VideoReadFile", "VideoSample", "VideoShow", "VideoWriteFile",
           "VideoReadWebcam", "read_y4m", "write_y4m", "iter_video_frames"]


# ---- Y4M codec (YUV4MPEG2) ------------------------------------------------------------------

def _yuv_to_rgb(y, u, v):
    y = y.astype(np.float32)
    u = u.astype(np.float32) - 128.0
    v = v.astype(np.float32) - 128.0
    r = y + 1.402 * v
    g = y - 0.344136 * u - 0.714136 * v
    b = y + 1.772 * u
    return np.clip(np.stack([r, g, b], -1) + 0.5, 0, 255).astype(np.uint8)


def _rgb_to_yuv(rgb):
    f = rgb.astype(np.float32)
    r, g, b = f[..., 0], f[..., 1], f[..., 2]
    y = 0.299 * r + 0.587 * g + 0.114 * b
    u = -0.168736 * r - 0.331264 * g + 0.5 * b + 128.0
    v = 0.5 * r - 0.418688 * g - 0.081312 * b + 128.0
    c = lambda a: np.clip(a + 0.5, 0, 255).astype(np.uint8)  # noqa: E731
    return c(y), c(u), c(v)


def iter_y4m(path):
    with open(path, "rb") as f:
        header = f.readline().decode("ascii").split()
        if not header or header[0] != "YUV4MPEG2":
            raise ValueError(f"{path}: not a YUV4MPEG2 file")
        params = {t[0]: t[1:] for t in header[1:]}
        w, h = int(params["W"]), int(params["H"])
        cs = params.get("C", "420jpeg")
        chroma444 = cs.startswith("444")
        cw, ch = (w, h) if chroma444 else ((w + 1) // 2, (h + 1) // 2)
        while True:
            line = f.readline()
            if not line:
                return
            if not line.startswith(b"FRAME"):
                raise ValueError(f"{path}: corrupt frame header")
            y = np.frombuffer(f.read(w * h), np.uint8).reshape(h, w)
            u = np.frombuffer(f.read(cw * ch), np.uint8).reshape(ch, cw)
            v = np.frombuffer(f.read(cw * ch), np.uint8).reshape(ch, cw)
            if not chroma444:
                u = u.repeat(2, 0).repeat(2, 1)[:h, :w]
                v = v.repeat(2, 0).repeat(2, 1)[:h, :w]
            yield _yuv_to_rgb(y, u, v)


def read_y4m(path) -> np.ndarray:
    return np.stack(list(iter_y4m(path)))


class Y4MWriter:
    def __init__(self, path, width, height, fps=30):
        self.f = open(path, "wb")
        self.w, self.h = width, height
        self.f.write(f"YUV4MPEG2 W{width} H{height} F{int(fps)}:1 Ip A1:1 C444\n".encode())

    def write(self, rgb):
        y, u, v = _rgb_to_yuv(np.asarray(rgb)[: self.h, : self.w])
        self.f.write(b"FRAME\n")
        self.f.write(y.tobytes())
        self.f.write(u.tobytes())
        self.f.write(v.tobytes())

    def close(self):
        self.f.close()


def write_y4m(path, frames, fps=30):
    frames = list(frames)
    h, w = frames[0].shape[:2]
    wr = Y4MWriter(path, w, h, fps)
    for fr in frames:
        wr.write(fr)
    wr.close()


def iter_video_frames(path):
    """RGB uint8 frames of a video file / frame directory, whatever backend is available."""
    path = Path(path)
    if path.is_dir():
        from PIL import Image
        for p in sorted(path.iterdir()):
            if p.suffix.lower() in (".png", ".jpg", ".jpeg", ".bmp", ".ppm"):
                yield np.asarray(Image.open(p).convert("RGB"))
        return
    suffix = path.suffix.lower()
    if suffix == ".avi" and not _CV2:
        yield from iter_avi(path)
    elif suffix == ".gif":
        from PIL import Image, ImageSequence
        with Image.open(path) as im:
            for fr in ImageSequence.Iterator(im):
                yield np.asarray(fr.convert("RGB"))
    elif suffix == ".y4m":
        yield from iter_y4m(path)
    elif suffix in (".npy", ".npz"):
        arr = np.load(path, allow_pickle=False)
        if hasattr(arr, "files"):
            arr = arr[arr.files[0]]
        yield from arr
    elif _CV2:
        cap = cv2.VideoCapture(str(path))
        if not cap.isOpened():
            raise ValueError(f"Couldn't open video file: {path}")
        try:
            while True:
                ok, bgr = cap.read()
                if not ok:
                    return
                yield cv2.cvtColor(bgr, cv2.COLOR_BGR2RGB)
        finally:
            cap.release()
    else:
        raise ValueError(f"{path}: unsupported video format without OpenCV "
                         f"(use .avi, .gif, .y4m, .npy or a frame directory)")


# ---- elements -------------------------------------------------------------------------------

class VideoOutput(PipelineElement):
    def __init__(self, context):
        context.set_protocol("video_output:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, images):
        return StreamEvent.OKAY, {"images": images}


class VideoReadFile(DataSource):
    def __init__(self, context):
        context.set_protocol("video_read_file:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def start_stream(self, stream, stream_id):
        stream.variables["video_frame_generator"] = None
        return super().start_stream(stream, stream_id, use_create_frame=False)

    def frame_generator(self, stream, frame_id):
        gen = stream.variables.get("video_frame_generator")
        while True:
            if gen is None:
                try:
                    path, _ = next(stream.variables["source_paths_generator"])
                except StopIteration:
                    return StreamEvent.STOP, {"diagnostic": "End of video file(s)"}
                try:
                    gen = iter_video_frames(path)
                except ValueError as exc:
                    return StreamEvent.ERROR, {"diagnostic": str(exc)}
                stream.variables["video_frame_generator"] = gen
            try:
                return StreamEvent.OKAY, {"images": [next(gen)]}
            except StopIteration:
                gen = None
                stream.variables["video_frame_generator"] = None
            except ValueError as exc:
                return StreamEvent.ERROR, {"diagnostic": str(exc)}

    def process_frame(self, stream, images):
        return StreamEvent.OKAY, {"images": images}

    def stop_stream(self, stream, stream_id):
        stream.variables["video_frame_generator"] = None
        return StreamEvent.OKAY, {}


class VideoSample(PipelineElement):
    def __init__(self, context):
        context.set_protocol("video_sample:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, images):
        rate, _ = self.get_parameter("sample_rate", 1)
        if stream.frame_id % int(rate):
            return StreamEvent.DROP_FRAME, {}
        return StreamEvent.OKAY, {"images": images}


class VideoShow(PipelineElement):
    def __init__(self, context):
        context.set_protocol("video_show:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, images):
        title, _ = self.get_parameter("title", "Video")
        for image in images:
            arr = np.asarray(image)
            if _CV2:
                try:
                    bgr = cv2.cvtColor(arr, cv2.COLOR_RGB2BGR) if arr.ndim == 3 else arr
                    cv2.imshow(title, bgr)
                    if cv2.waitKey(1) & 0xFF == ord("x"):
                        return StreamEvent.STOP, {"diagnostic": "VideoShow exit"}
                    continue
                except Exception:
                    pass
            self.logger.debug(f"{title} {self.my_id()}: {arr.shape} mean={float(arr.mean()):.1f}")
        return StreamEvent.OKAY, {}

    def stop_stream(self, stream, stream_id):
        if _CV2:
            try:
                cv2.destroyAllWindows()
            except Exception:
                pass
        return StreamEvent.OKAY, {}


class VideoWriteFile(DataTarget):
    """Writes ``.avi`` (parameters ``codec``: ``MJPG`` (default) | ``raw``, ``quality``),
    ``.gif``, ``.y4m`` or ``.npy``; other suffixes need OpenCV.  ``rate``: frames per second."""

    def __init__(self, context):
        context.set_protocol("video_write_file:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def start_stream(self, stream, stream_id):
        event, diag = super().start_stream(stream, stream_id)
        if event == StreamEvent.OKAY:
            path = stream.variables["target_path"]
            if contains_all(path, "{}"):
                path = path.format(stream.variables["target_file_id"])
            stream.variables["video_path"] = path
            stream.variables["video_writer"] = None
            stream.variables["video_frames"] = []
        return event, diag

    def process_frame(self, stream, images):
        path = stream.variables["video_path"]
        suffix = Path(path).suffix.lower()
        for image in images:
            arr = np.asarray(image).astype(np.uint8)
            if suffix in (".npy", ".gif"):
                stream.variables["video_frames"].append(arr)
                continue
            writer = stream.variables["video_writer"]
            if writer is None:
                rate, _ = self.get_parameter("rate", 30)
                if suffix == ".y4m":
                    writer = Y4MWriter(path, arr.shape[1], arr.shape[0], float(rate))
                elif suffix == ".avi" and not _CV2:
                    codec, _ = self.get_parameter("codec", "MJPG")
                    quality, _ = self.get_parameter("quality", 90)
                    writer = AviWriter(path, arr.shape[1], arr.shape[0], float(rate), str(codec), int(quality))
                elif _CV2:
                    writer = cv2.VideoWriter(path, cv2.VideoWriter_fourcc(*"mp4v"), float(rate),
                                             (arr.shape[1], arr.shape[0]))
                else:
                    return StreamEvent.ERROR, {"diagnostic": f"{path}: unsupported format without OpenCV"}
                stream.variables["video_writer"] = writer
            if isinstance(writer, (Y4MWriter, AviWriter)):
                writer.write(arr)
            else:
                writer.write(cv2.cvtColor(arr, cv2.COLOR_RGB2BGR))
        return StreamEvent.OKAY, {}

    def stop_stream(self, stream, stream_id):
        path = stream.variables.get("video_path")
        frames = stream.variables.get("video_frames")
        suffix = Path(path).suffix.lower() if path else ""
        if path and frames and suffix == ".npy":
            np.save(path, np.stack(frames))
        elif path and frames and suffix == ".gif":
            from PIL import Image
            rate, _ = self.get_parameter("rate", 30)
            ims = [Image.fromarray(f if f.ndim == 3 else np.repeat(f[..., None], 3, 2)) for f in frames]
            ims[0].save(path, save_all=True, append_images=ims[1:], duration=int(round(1000 / float(rate))), loop=0)
        writer = stream.variables.get("video_writer")
        if writer is not None:
            (writer.close if isinstance(writer, (Y4MWriter, AviWriter)) else writer.release)()
        return StreamEvent.OKAY, {}


from .webcam_io import VideoReadWebcam  # noqa: E402,F401  (kept importable from here)
