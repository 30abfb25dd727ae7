"""YoloDetector example element with the reference's interface (``examples/yolo/yolo.py:46-87``):
``images`` (list of HxWx3 uint8 RGB arrays, or a uint8 device batch) -> ``overlay`` =
``{"objects": [{"name", "confidence"}], "rectangles": [{"x", "y", "w", "h"}]}``.

Instead of Ultralytics on one image at a time, same-sized images are stacked into one batch,
uploaded once (pinned staging) and run through :class:`~aiko_services_amd.models.yolov8.YOLOv8`
on the HIP kernels (letterbox, network, DFL decode and NMS all on the GPU); only the fixed-size
detection rows come back.  Weights are random-init (the reference's custom
``yolov8n_robotdog.pt`` is not available), so detections are structural, not semantic.
Parameters: ``scale`` (n/s/m/l/x), ``conf``, ``iou``, ``class_filter`` (list of class ids,
default all), ``image_size`` (640).
"""
from __future__ import annotations

import numpy as np
import torch

from aiko_services_amd.gpu.element import GpuPipelineElement
from aiko_services_amd.pipeline.stream import StreamEvent
from aiko_services_amd.utils.sexpr import parse

__all__ = ["YoloDetector", "COCO_NAMES"]

COCO_NAMES = (
    "person bicycle car motorcycle airplane bus train truck boat traffic_light fire_hydrant "
    "stop_sign parking_meter bench bird cat dog horse sheep cow elephant bear zebra giraffe "
    "backpack umbrella handbag tie suitcase frisbee skis snowboard sports_ball kite baseball_bat "
    "baseball_glove skateboard surfboard tennis_racket bottle wine_glass cup fork knife spoon bowl "
    "banana apple sandwich orange broccoli carrot hot_dog pizza donut cake chair couch potted_plant "
    "bed dining_table toilet tv laptop mouse remote keyboard cell_phone microwave oven toaster sink "
    "refrigerator book clock vase scissors teddy_bear hair_drier toothbrush").split()


class YoloDetector(GpuPipelineElement):
    PROTOCOL = "object_detector:0"

    def __init__(self, context):
        context.set_protocol(self.PROTOCOL)
        super().__init__(context)
        self.model = None
        self._pinned = {}

    def _ensure_model(self):
        if self.model is None:
            from aiko_services_amd.models.yolov8 import YOLOv8
            from aiko_services_amd.ops import require_native
            require_native()
            p = lambda n, d: self.get_parameter(n, d)[0]  # noqa: E731
            self.model = YOLOv8(scale=str(p("scale", "n")), device=self.device,
                                image_size=int(p("image_size", 640)), conf=float(p("conf", 0.25)),
                                iou=float(p("iou", 0.7)), max_det=int(p("max_det", 300)))
            self.load_model_weights(self.model)
        return self.model

    def start_stream(self, stream, stream_id):
        self._ensure_model()
        return StreamEvent.OKAY, {}

    def _class_filter(self):
        value, found = self.get_parameter("class_filter", None)
        if not found or value in (None, "", "all"):
            return None
        if isinstance(value, str):
            _, items = parse(value) if value.startswith("(") else (None, value.split())
            value = items
        return {int(v) for v in value}

    def _batches(self, images):
        if isinstance(images, torch.Tensor):
            yield images if images.dim() == 4 else images[None]
            return
        groups: dict = {}
        for img in images:
            a = np.asarray(img, dtype=np.uint8)
            groups.setdefault(a.shape, []).append(a)
        for shape, arrs in groups.items():
            host = self._pinned.get((len(arrs), shape))
            if host is None:
                host = torch.empty((len(arrs),) + shape, dtype=torch.uint8,
                                   pin_memory=self.device.type == "cuda")
                self._pinned[(len(arrs), shape)] = host
            host.copy_(torch.from_numpy(np.stack(arrs)))
            yield host.to(self.device, non_blocking=True)

    def process_frame(self, stream, images):
        model = self._ensure_model()
        keep = self._class_filter()
        overlay = {"objects": [], "rectangles": []}
        for batch in self._batches(images):
            det, count = model.detect(batch.contiguous())
            det, count = det.cpu(), count.cpu()
            for b in range(det.shape[0]):
                for x1, y1, x2, y2, score, cls in det[b, :int(count[b])].tolist():
                    c = int(cls)
                    if keep is not None and c not in keep:
                        continue
                    name = COCO_NAMES[c] if c < len(COCO_NAMES) else f"class_{c}"
                    overlay["objects"].append({"name": name, "confidence": round(score, 2)})
                    overlay["rectangles"].append({"x": int(x1), "y": int(y1), "w": int(x2 - x1), "h": int(y2 - y1)})
        return StreamEvent.OKAY, {"overlay": overlay}
