"""Robot controller Actor (reference ``examples/xgo_robot/robot_control.py:84-295``).

Subscribes to the robot's binary video topic (``zlib(np.save(image))`` payloads, the
reference's off-node data path), keeps the latest frame and a frame count in its EC share, and
optionally runs a detector on each frame: ``detector="yolo"`` uses the GPU ``YOLOv8`` model on
the HIP kernels and publishes ``(detections frame_id (name confidence x y w h) ...)`` on
``{namespace}/detections``.  Robot commands go through a remote proxy of the ``XGORobot``
interface (``get_actor_mqtt``), e.g. ``control.robot("turn", 30)``.

    python -m aiko_services_amd.examples.xgo_robot.robot_control --robot <robot /in topic>
"""
from __future__ import annotations

from abc import abstractmethod
import argparse
import time

import numpy as np

import aiko_services_amd as aiko
from aiko_services_amd.runtime.actor import Actor
from aiko_services_amd.runtime.context import Interface
from aiko_services_amd.runtime.process import aiko as _aiko
from aiko_services_amd.utils.configuration import get_namespace
from aiko_services_amd.utils.sexpr import generate

from aiko_services_amd.runtime import event

from .xgo_robot import XGORobot, topic_video, video_frame, video_payload

__all__ = ["RobotControl", "RobotControlImpl", "VideoTest", "VideoTestImpl"]

SLEEP_PERIOD = 0.2          # seconds between published frames (EC-tunable ``sleep_period``)


class RobotControl(Actor):
    Interface.default("RobotControl", "aiko_services_amd.examples.xgo_robot.robot_control.RobotControlImpl")

    @abstractmethod
    def robot(self, command, *args): ...


class RobotControlImpl(RobotControl):
    def __init__(self, context, robot_topic=None, detector=None):
        context.get_implementation("Actor").__init__(self, context)
        self.robot_topic = robot_topic
        self.detector = detector
        self._model = None
        self.last_image = None
        self.share.update({"frames_received": 0, "robot_topic": robot_topic or "", "detections": 0})
        _aiko.process.add_message_handler(self._video_handler, topic_video(), binary=True)

    def _video_handler(self, _aiko_ctx, topic, payload):
        image = video_frame(payload)
        if image is None:                 # frame-ring slot reused before we read it: dropped
            return True
        self.last_image = image
        n = int(self.share["frames_received"]) + 1
        self.ec_producer.update("frames_received", n)
        if self.detector == "yolo":
            self._detect(n, image)
        return True

    def _detect(self, frame_id, image):
        import torch
        if self._model is None:
            from aiko_services_amd.models.yolov8 import YOLOv8
            self._model = YOLOv8(scale="n", device="cuda", image_size=640)
        det, count = self._model.detect(torch.from_numpy(image)[None].cuda())
        rows = det[0, :int(count[0])].tolist()
        items = [[f"class_{int(c)}", f"{s:.2f}", int(x1), int(y1), int(x2 - x1), int(y2 - y1)]
                 for x1, y1, x2, y2, s, c in rows]
        self.ec_producer.update("detections", int(self.share["detections"]) + len(items))
        _aiko.message.publish(f"{get_namespace()}/detections", generate("detections", [frame_id] + items))

    def robot(self, command, *args):
        """Forward one XGORobot method call to the robot actor's /in topic."""
        if not self.robot_topic:
            return
        proxy = aiko.get_actor_mqtt(self.robot_topic, XGORobot)
        getattr(proxy, command)(*args)


class VideoTest(Actor):
    """Video source for testing the controller without a robot (reference
    ``robot_control.py:302-355``): publishes ``zlib(np.save(image))`` frames on the video topic
    every ``sleep_period`` seconds.  The reference reads camera 0 through OpenCV; without a
    camera (no OpenCV in this image) frames are a synthetic moving gradient, 240 x 320 RGB, with
    the per-frame time and rate in the share instead of drawn into the image."""
    Interface.default("VideoTest", "aiko_services_amd.examples.xgo_robot.robot_control.VideoTestImpl")


class VideoTestImpl(VideoTest):
    def __init__(self, context, size=(240, 320)):
        context.get_implementation("Actor").__init__(self, context)
        self.size = (int(size[0]), int(size[1]))
        self.share.update({"sleep_period": SLEEP_PERIOD, "source_file": __file__, "topic_video": topic_video(),
                           "frames_published": 0, "fps": 0, "time_process_ms": 0.0})
        self._frame_id = 0
        self._last = None
        self._period = None
        self._schedule()

    def _schedule(self):
        try:
            period = float(self.share["sleep_period"])
        except (TypeError, ValueError):
            period = SLEEP_PERIOD
        period = max(period, 0.001)
        if period != self._period:                 # live retune via (update sleep_period ...)
            if self._period is not None:
                event.remove_timer_handler(self._tick)
            event.add_timer_handler(self._tick, period)
            self._period = period

    def frame(self) -> np.ndarray:
        h, w = self.size
        yy, xx = np.mgrid[0:h, 0:w]
        k = self._frame_id
        image = np.stack([(xx + 4 * k) % 256, (yy + 2 * k) % 256, np.full_like(xx, (16 * k) % 256)], axis=-1)
        return image.astype(np.uint8)

    def _tick(self):
        t0 = time.time()
        image = self.frame()
        self.share["time_process_ms"] = round((time.time() - t0) * 1000, 1)
        _aiko.message.publish(self.share["topic_video"], video_payload(image))
        self._frame_id += 1
        self.ec_producer.update("frames_published", self._frame_id)
        if self._last is not None:
            self.share["fps"] = int(1.0 / max(t0 - self._last, 1e-6))
        self._last = t0
        self._schedule()


def main(argv=None):
    ap = argparse.ArgumentParser(description="robot controller actor (or --video_test: test video source)")
    ap.add_argument("--robot", default=None, help="robot actor /in topic")
    ap.add_argument("--detector", default=None, choices=[None, "yolo"])
    ap.add_argument("--video_test", action="store_true", help="run the VideoTest source instead")
    a = ap.parse_args(argv)
    if a.video_test:
        aiko.compose_instance(VideoTestImpl, aiko.actor_args("video_test"))
    else:
        args = aiko.actor_args("robot_control")
        args.update(robot_topic=a.robot, detector=a.detector)
        aiko.compose_instance(RobotControlImpl, args)
    aiko.process.run()


if __name__ == "__main__":
    main()
