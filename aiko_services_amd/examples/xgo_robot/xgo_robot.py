"""XGO robot-dog Actor (reference ``examples/xgo_robot/xgo_robot.py:109-411``), simulated.

The ``XGORobot`` interface keeps the reference's remote methods — ``action``, ``arm``,
``arm_mode``, ``attitude``, ``body_mode``, ``claw``, ``move``, ``reset``, ``screen_detail``,
``stop``, ``terminate``, ``translation``, ``turn`` — callable as S-expressions on the actor's
``/in`` topic (e.g. ``(turn 30)``).  There is no robot, serial port or camera here, so
``XGORobotImpl`` integrates the commanded motion into a simulated pose published in its EC
share (``pose``, ``claw``, ``arm``, ``attitude`` ...) and its "camera" publishes synthetic RGB
frames on ``{namespace}/video`` as the reference does: ``zlib(np.save(image))`` binary payloads
(``parameters``: ``fps``, ``width``, ``height``).

    python -m aiko_services_amd.examples.xgo_robot.xgo_robot [--fps 5]
"""
from __future__ import annotations

from abc import abstractmethod
import argparse
from io import BytesIO
import math
import os
import zlib

import numpy as np

import aiko_services_amd as aiko
from aiko_services_amd.runtime import event
from aiko_services_amd.runtime.actor import Actor
from aiko_services_amd.runtime.context import Interface
from aiko_services_amd.runtime.process import aiko as _aiko
from aiko_services_amd.utils.configuration import get_namespace

__all__ = ["XGORobot", "XGORobotImpl", "encode_image", "decode_image", "video_payload", "video_frame",
           "topic_video", "ACTIONS"]

ACTIONS = {"lie_down": 1, "stand_up": 2, "crawl": 3, "turn_around": 4, "mark_time": 5, "squat": 6,
           "turn_roll": 7, "turn_pitch": 8, "turn_yaw": 9, "three_axis": 10, "pee": 11, "sit_down": 12,
           "wave": 13, "stretch": 14, "wave_body": 15, "swing": 16, "pray": 17, "seek": 18,
           "handshake": 19, "play_ball": 20}
LIMITS = {"arm_x": (-80, 155), "arm_z": (-95, 155), "pitch": (-15, 15), "roll": (-20, 10),
          "yaw": (-11, 11), "stride_x": (-25, 25), "stride_y": (-18, 18), "turn": (-100, 100),
          "tx": (-35, 35), "ty": (-18, 18), "tz": (75, 115), "claw": (0, 255)}


def topic_video() -> str:
    return f"{get_namespace()}/video"


def encode_image(image: np.ndarray) -> bytes:
    buf = BytesIO()
    np.save(buf, np.asarray(image), allow_pickle=False)
    return zlib.compress(buf.getvalue(), 1)


def decode_image(payload: bytes) -> np.ndarray:
    return np.load(BytesIO(zlib.decompress(payload)), allow_pickle=False)


_RING = None


def video_payload(image: np.ndarray):
    """What to publish for one video frame: the reference's ``zlib(np.save(image))`` bytes, or
    — with ``AIKO_FRAME_RING=1`` (publisher and subscribers on one node) — a slot token of a
    shared-memory frame ring (``message/frame_ring.py``): the pixels never cross the broker."""
    global _RING
    if os.environ.get("AIKO_FRAME_RING", "0") in ("1", "true"):
        if _RING is None:
            from ...message.frame_ring import SharedFrameRing
            _RING = SharedFrameRing(f"aiko_video_{os.getpid()}", slots=16,
                                    slot_bytes=max(np.asarray(image).nbytes, 1 << 16), create=True)
        return _RING.put(image)
    return encode_image(image)


def video_frame(payload):
    """Inverse of :func:`video_payload` (None if a ring slot was overwritten before the read)."""
    from ...message.frame_ring import SharedFrameRing, is_ring_token
    if is_ring_token(payload):
        return SharedFrameRing.get(payload)
    return decode_image(payload)


def _clip(name, value):
    lo, hi = LIMITS[name]
    return max(lo, min(hi, float(value)))


def _given(v):
    return v is not None and str(v) != "nil"


class XGORobot(Actor):
    Interface.default("XGORobot", "aiko_services_amd.examples.xgo_robot.xgo_robot.XGORobotImpl")

    @abstractmethod
    def action(self, value): ...

    @abstractmethod
    def arm(self, x, z): ...

    @abstractmethod
    def arm_mode(self, stabilize): ...

    @abstractmethod
    def attitude(self, pitch="nil", roll="nil", yaw="nil"): ...

    @abstractmethod
    def body_mode(self, stabilize): ...

    @abstractmethod
    def claw(self, grip): ...

    @abstractmethod
    def move(self, direction, stride="nil"): ...

    @abstractmethod
    def reset(self): ...

    @abstractmethod
    def screen_detail(self, enabled=None): ...

    @abstractmethod
    def stop(self): ...

    @abstractmethod
    def terminate(self, immediate=False): ...

    @abstractmethod
    def translation(self, x="nil", y="nil", z="nil"): ...

    @abstractmethod
    def turn(self, speed): ...


class XGORobotImpl(XGORobot):
    def __init__(self, context, fps: float = 5.0, width: int = 320, height: int = 240):
        context.get_implementation("Actor").__init__(self, context)
        self.fps, self.size = float(fps), (int(height), int(width))
        self._velocity = [0.0, 0.0]        # mm per tick along x / y
        self._turn_rate = 0.0              # degrees per second
        self._frame_id = 0
        self._rng = np.random.default_rng(0)
        self.share.update({"battery": 100, "screen_detail": False, "topic_video": topic_video(),
                           "version_firmware": "simulated", "action": "none", "claw": 0,
                           "arm": [0, 0], "arm_stabilize": False, "body_stabilize": False,
                           "attitude": [0, 0, 0], "translation": [0, 0, 105], "pose": [0.0, 0.0, 0.0],
                           "frames_published": 0})
        if self.fps > 0:
            event.add_timer_handler(self._tick, 1.0 / self.fps)

    # ---- simulation ---------------------------------------------------------------------------
    def _tick(self):
        x, y, heading = self.share["pose"]
        heading = (heading + self._turn_rate / self.fps) % 360.0
        rad = math.radians(heading)
        vx, vy = self._velocity
        x += vx * math.cos(rad) - vy * math.sin(rad)
        y += vx * math.sin(rad) + vy * math.cos(rad)
        self.share["pose"] = [round(x, 2), round(y, 2), round(heading, 2)]
        h, w = self.size
        image = self._rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        image[:8, :8] = self._frame_id % 256                    # frame stamp for consumers
        _aiko.message.publish(topic_video(), video_payload(image))
        self._frame_id += 1
        self.ec_producer.update("frames_published", self._frame_id)

    # ---- XGORobot -----------------------------------------------------------------------------
    def action(self, value):
        if value in ACTIONS:
            self.ec_producer.update("action", value)

    def arm(self, x, z):
        self.ec_producer.update("arm", [_clip("arm_x", x), _clip("arm_z", z)])

    def arm_mode(self, stabilize):
        self.ec_producer.update("arm_stabilize", str(stabilize).lower() == "true")

    def attitude(self, pitch="nil", roll="nil", yaw="nil"):
        p, r, y = self.share["attitude"]
        self.ec_producer.update("attitude", [_clip("pitch", pitch) if _given(pitch) else p,
                                             _clip("roll", roll) if _given(roll) else r,
                                             _clip("yaw", yaw) if _given(yaw) else y])

    def body_mode(self, stabilize):
        self.ec_producer.update("body_stabilize", str(stabilize).lower() == "true")

    def claw(self, grip):
        self.ec_producer.update("claw", int(_clip("claw", grip)))

    def move(self, direction, stride="nil"):
        stride = float(stride) if _given(stride) else 0.0
        if direction == "x":
            self._velocity[0] = _clip("stride_x", stride)
        elif direction == "y":
            self._velocity[1] = _clip("stride_y", stride)

    def reset(self):
        self.stop()
        self.share.update({"action": "none", "claw": 0, "arm": [0, 0], "attitude": [0, 0, 0],
                           "translation": [0, 0, 105]})

    def screen_detail(self, enabled=None):
        value = (not self.share["screen_detail"]) if enabled is None else str(enabled).lower() == "true"
        self.ec_producer.update("screen_detail", value)

    def stop(self):
        self._velocity = [0.0, 0.0]
        self._turn_rate = 0.0

    def terminate(self, immediate=False):
        self.stop()
        if self.fps > 0:
            event.remove_timer_handler(self._tick)
        aiko.process.terminate()

    def translation(self, x="nil", y="nil", z="nil"):
        tx, ty, tz = self.share["translation"]
        self.ec_producer.update("translation", [_clip("tx", x) if _given(x) else tx,
                                                _clip("ty", y) if _given(y) else ty,
                                                _clip("tz", z) if _given(z) else tz])

    def turn(self, speed):
        self._turn_rate = _clip("turn", speed)


def main(argv=None):
    ap = argparse.ArgumentParser(description="simulated XGO robot actor")
    ap.add_argument("--fps", type=float, default=5.0)
    a = ap.parse_args(argv)
    args = aiko.actor_args("xgo_robot")
    args["fps"] = a.fps
    robot = aiko.compose_instance(XGORobotImpl, args)
    print(f"MQTT topic: {robot.topic_in}", flush=True)
    aiko.process.run()


if __name__ == "__main__":
    main()
