"""bench.py's per-model defaults (the driver runs it with only --gpus/--steps/--warmup): the
batch sizes chosen for tile quantisation on 256 CUs and the configs' frame sizes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_resnet_default_batch_fills_the_chip():
    a = bench.parse_args(["--gpus", "1", "--steps", "20", "--warmup", "5"])
    assert a.model == "resnet50" and a.batch == 640 and (a.height, a.width) == (224, 224)
    # stage 3 (14 x 14 outputs) at 256-row tiles: whole rounds over 256 CUs, >= 95 % busy
    tiles = -(-a.batch * 196 // 256)
    rounds = -(-tiles // 256)
    assert tiles / (256 * rounds) >= 0.95


def test_model_defaults_and_explicit_overrides():
    assert bench.parse_args(["--model", "yolov8n"]).batch == 192
    y = bench.parse_args(["--model", "yolov8n"])
    assert (y.height, y.width) == (480, 640)
    assert bench.parse_args(["--model", "whisper-small"]).batch == 28
    assert bench.parse_args(["--batch", "256"]).batch == 256
    p = bench.parse_args(["--parallel", "pp", "--height", "224", "--width", "224"])
    assert (p.height, p.width) == (224, 224) and p.batch == 640
    assert (bench.parse_args(["--parallel", "pp"]).height, bench.parse_args([]).height) == (480, 224)
