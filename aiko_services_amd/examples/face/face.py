"""FaceDetector example element with the reference's interface (``examples/face/face.py:45-80``):
``images`` (list of HxWx3 uint8 RGB arrays or a uint8 device batch) -> ``overlay`` =
``{"rectangles": [{"x", "y", "w", "h"}]}``; the EC share keeps a running ``detections`` count.

The reference calls DeepFace's RetinaFace one image at a time on the CPU.  Here a single-class
YOLOv8 detector ("covered by the K4 conv / NMS kernels") runs the whole batch on
the HIP kernels — letterbox, network, DFL decode and NMS on the GPU.  Weights are random-init
unless a ``weights`` file is given, so detections are structural, not semantic.
Parameters: ``scale`` (n), ``conf`` (0.25), ``iou`` (0.5), ``image_size`` (640), ``weights``.
"""
from __future__ import annotations

from aiko_services_amd.examples.yolo.yolo import YoloDetector
from aiko_services_amd.pipeline.stream import StreamEvent

__all__ = ["FaceDetector"]


class FaceDetector(YoloDetector):
    PROTOCOL = "face_detector:0"

    def __init__(self, context):
        super().__init__(context)
        self.share["detections"] = 0

    def _ensure_model(self):
        if self.model is None:
            from aiko_services_amd.models.yolov8 import YOLOv8
            from aiko_services_amd.ops import require_native
            require_native()
            p = lambda n, d: self.get_parameter(n, d)[0]  # noqa: E731
            self.model = YOLOv8(scale=str(p("scale", "n")), num_classes=1, device=self.device,
                                image_size=int(p("image_size", 640)), conf=float(p("conf", 0.25)),
                                iou=float(p("iou", 0.5)), max_det=int(p("max_det", 300)))
            self.load_model_weights(self.model)
        return self.model

    def process_frame(self, stream, images):
        event, out = super().process_frame(stream, images)
        rects = out["overlay"]["rectangles"]
        if rects:
            self.ec_producer.update("detections", int(self.share["detections"]) + len(rects))
        return event, {"overlay": {"rectangles": rects}}
