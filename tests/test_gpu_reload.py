"""a hipGraph captured before ``load_state_dict`` must replay the NEW weights —
including the derived stem images (ResNet fused stem+pool, YOLO direct stem), which are
rebuilt into their existing tensors rather than re-allocated."""
import pytest
import torch

from aiko_services_amd.gpu.element import CapturedCall

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _frames(B, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, generator=g).to(DEV)


@pytest.mark.parametrize("model", ["resnet50", "yolov8n"])
def test_captured_graph_sees_reloaded_weights(native, model):
    if model == "resnet50":
        from aiko_services_amd.models.resnet50 import ResNet50
        a, b = ResNet50(seed=0, device=DEV), ResNet50(seed=1, device=DEV)
        x = _frames(2, 224, 224)
        run = lambda t: a.logits(t)
    else:
        from aiko_services_amd.models.yolov8 import YOLOv8
        a, b = YOLOv8(scale="n", seed=0, device=DEV), YOLOv8(scale="n", seed=1, device=DEV)
        x = _frames(2, 480, 640)
        run = lambda t: a.head_outputs(None, a0=a.stem_from_frames(t))[0]
    run(x)                                   # eager first (derived images get built)
    call = CapturedCall(run, [x])
    before = call(x).clone()
    a.load_state_dict(b.state_dict())        # in-place copy of different weights
    replay = call(x).clone()
    eager = run(x).clone()
    torch.cuda.synchronize()
    assert not torch.equal(before, replay), "replay still uses the old weights"
    assert torch.equal(replay, eager)
