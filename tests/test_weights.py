"""Weight persistence: packed bf16 conv weights, fp8 weights + scale tables,
safetensors files with the model config in the metadata, derived (fused) layers re-built."""
import pytest
import torch

from aiko_services_amd.models import weights as Wt
from aiko_services_amd.models.resnet50 import ResNet50
from aiko_services_amd.models.whisper import WhisperEncoder
from aiko_services_amd.models.yolov8 import YOLOv8

CASES = [(ResNet50, {}), (YOLOv8, {"scale": "n"}), (WhisperEncoder, {"size": "tiny"})]


def _same(a: dict, b: dict):
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("cls,kw", CASES, ids=lambda c: getattr(c, "__name__", ""))
def test_save_load_roundtrip(cls, kw, tmp_path):
    a = cls(seed=0, device="cpu", **kw)
    b = cls(seed=1, device="cpu", **kw)
    path = str(tmp_path / "w.safetensors")
    a.save(path, with_reference=True)
    meta = Wt.read_metadata(path)
    assert meta["model"] == cls.__name__ and meta["config"] == a.config()
    b.load(path)
    _same(a.state_dict(with_reference=True), b.state_dict(with_reference=True))
    # derived layers follow their sources
    if cls is ResNet50:
        for x, y in zip(a.blocks, b.blocks):
            if x.fused is not None:
                assert torch.equal(x.fused.weight, y.fused.weight) and torch.equal(x.fused.bias, y.fused.bias)
    if cls is YOLOv8:
        for x, y in zip(a.heads, b.heads):
            assert torch.equal(x.first.weight, y.first.weight) and torch.equal(x.first.bias, y.first.bias)
    # a dict without fp32 references drops them (they would be stale)
    c = cls(seed=2, device="cpu", **kw)
    c.load_state_dict(a.state_dict())
    name, layer = next(iter(c.named_layers()))
    assert layer.ref_weight is None


def test_load_rejects_mismatch(tmp_path):
    y = YOLOv8(scale="n", device="cpu")
    path = str(tmp_path / "y.safetensors")
    y.save(path)
    with pytest.raises(ValueError):
        ResNet50(device="cpu").load(path)
    with pytest.raises(ValueError):          # same class, different width
        YOLOv8(scale="s", device="cpu").load(path)
    sd = y.state_dict()
    sd.pop(next(iter(sd)))
    with pytest.raises(KeyError):
        YOLOv8(scale="n", device="cpu").load_state_dict(sd)
    assert YOLOv8(scale="n", device="cpu").load_state_dict(sd, strict=False)
