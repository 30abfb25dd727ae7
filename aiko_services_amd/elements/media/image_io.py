"""Image elements (reference ``elements/media/image_io.py:82-255``), PIL/numpy based.

OpenCV is not available on the MI355X boxes, so overlays are drawn with PIL and resizing
uses PIL on the host — or, when the images are a GPU uint8 batch tensor ``[B, H, W, 3]``, the
fused HIP resize kernel (``ops.preprocess`` path) via :class:`ImageResize` parameter
``device``.
"""
from __future__ import annotations

import numpy as np

from ...pipeline.engine import PipelineElement
from ...pipeline.stream import StreamEvent
from .common_io import DataSource, DataTarget

try:
    from PIL import Image, ImageDraw
    _PIL = True
except ImportError:  # pragma: no cover
    _PIL = False

__all__ = ["ImageOutput", "ImageOverlay", "ImageReadFile", "ImageResize", "ImageSynthetic",
           "ImageWriteFile", "to_numpy_rgb"]


def to_numpy_rgb(image) -> np.ndarray:
    if isinstance(image, np.ndarray):
        return image
    if _PIL and isinstance(image, Image.Image):
        return np.asarray(image.convert("RGB"))
    if hasattr(image, "detach"):  # torch tensor
        return image.detach().cpu().numpy()
    raise TypeError(f"unsupported image type {type(image).__name__}")


class ImageOutput(PipelineElement):
    def __init__(self, context):
        context.set_protocol("image_output:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, images):
        return StreamEvent.OKAY, {"images": images}


class ImageOverlay(PipelineElement):
    """Draw ``overlay["rectangles"]`` (x, y, w, h) with optional ``objects`` labels."""

    def __init__(self, context):
        context.set_protocol("image_overlay:0")
        context.get_implementation("PipelineElement").__init__(self, context)
        self.color = (0, 255, 255)
        self.thickness = 2
        self.threshold = 0.0

    def process_frame(self, stream, images, overlay):
        out = []
        for image in images:
            arr = to_numpy_rgb(image)
            gray = arr.ndim == 2
            pil = Image.fromarray(arr.astype(np.uint8)).convert("RGB")
            draw = ImageDraw.Draw(pil)
            rects = overlay.get("rectangles", []) if isinstance(overlay, dict) else []
            objects = overlay.get("objects", [{}] * len(rects)) if isinstance(overlay, dict) else []
            for obj, r in zip(objects, rects):
                conf = float(obj.get("confidence", 1.0))
                if conf <= self.threshold:
                    continue
                x, y, w, h = (int(float(r[k])) for k in ("x", "y", "w", "h"))
                draw.rectangle([x, y, x + w, y + h], outline=self.color, width=self.thickness)
                name = obj.get("name")
                if name:
                    ty = y - 12 if y > 14 else y + h + 2
                    draw.text((x, ty), f"{name}: {conf:0.2f}", fill=self.color)
            res = np.asarray(pil)
            out.append(res.mean(axis=2).astype(np.uint8) if gray else res)
        return StreamEvent.OKAY, {"images": out}


class ImageReadFile(DataSource):
    def __init__(self, context):
        context.set_protocol("image_read_file:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, paths):
        images = []
        for path in paths:
            try:
                images.append(Image.open(path))
            except Exception as exc:
                return StreamEvent.ERROR, {"diagnostic": f"Error loading image: {exc}"}
        return StreamEvent.OKAY, {"images": images}


class ImageSynthetic(PipelineElement):
    """Frame generator of random host images: parameters ``width`` / ``height`` (640 x 480),
    ``batch`` images per frame (1), ``limit`` frames (unbounded when absent), ``rate`` frames/s,
    ``seed``.  Stands in for a camera or video file where none is available (BASELINE frames
    are synthetic)."""

    def __init__(self, context):
        context.set_protocol("image_synthetic:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def start_stream(self, stream, stream_id):
        rate, _ = self.get_parameter("rate", default=None)
        self.create_frames(stream, self._generate, rate=float(rate) if rate else None)
        return StreamEvent.OKAY, {}

    def _generate(self, stream, frame_id):
        limit, found = self.get_parameter("limit")
        if found and limit is not None and frame_id >= int(limit):
            return StreamEvent.STOP, {"diagnostic": "frame limit reached"}
        w = int(self.get_parameter("width", 640)[0])
        h = int(self.get_parameter("height", 480)[0])
        n = int(self.get_parameter("batch", 1)[0])
        rng = np.random.default_rng(int(self.get_parameter("seed", 0)[0]) + frame_id)
        return StreamEvent.OKAY, {"images": [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for _ in range(n)]}

    def process_frame(self, stream, images):
        return StreamEvent.OKAY, {"images": images}


class ImageResize(PipelineElement):
    """``resolution`` = ``"WxH"``.  Host images (PIL / numpy) resize bilinearly on the CPU; a
    device uint8 batch ``[B, H, W, 3]`` is resized on the GPU by the HIP kernel."""

    def __init__(self, context):
        context.set_protocol("image_resize:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, images):
        resolution, found = self.get_parameter("resolution")
        if not found:
            return StreamEvent.ERROR, {"diagnostic": 'Must provide "resolution" parameter'}
        width, height = (int(v) for v in str(resolution).lower().split("x"))
        if hasattr(images, "is_cuda") and images.is_cuda:
            from ...ops.vision import resize_u8
            return StreamEvent.OKAY, {"images": resize_u8(images, (height, width))}
        out = []
        for image in images:
            if isinstance(image, np.ndarray):
                out.append(np.asarray(Image.fromarray(image).resize((width, height), Image.BILINEAR)))
            else:
                out.append(image.resize((width, height), Image.BILINEAR))
        return StreamEvent.OKAY, {"images": out}


class ImageWriteFile(DataTarget):
    def __init__(self, context):
        context.set_protocol("image_write_file:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, images):
        for image in images:
            path = self.next_target_path(stream)
            if not (_PIL and isinstance(image, Image.Image)):
                try:
                    image = Image.fromarray(to_numpy_rgb(image).astype("uint8"))
                except TypeError as exc:
                    return StreamEvent.ERROR, {"diagnostic": str(exc)}
            try:
                image.save(path)
            except Exception as exc:
                return StreamEvent.ERROR, {"diagnostic": f"Error saving image: {exc}"}
        return StreamEvent.OKAY, {}
