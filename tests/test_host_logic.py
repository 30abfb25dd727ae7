"""Host-side decision logic of the GPU paths (no GPU needed): which ResNet-50 block boundaries
the chained 1x1 kernel takes, Whisper token -> text rendering and the reference's speech reply
filter, the decode-attention workspace size, narrow-kernel eligibility, the host window shift."""
import torch

from aiko_services_amd.ops import conv as C


def _resnet_specs():
    """ResNet-50 bottleneck conv specs (CPU), as models/resnet50.py builds them."""
    g = torch.Generator().manual_seed(0)

    def conv(cout, cin, k, stride=1, act="relu"):
        return C.make_conv_spec(torch.randn(cout, cin, k, k, generator=g), torch.randn(cout, generator=g),
                                stride=stride, pad=k // 2, act=act)
    return conv


def test_chain_ok_shapes():
    conv = _resnet_specs()
    exp1, red1 = conv(256, 64, 1), conv(64, 256, 1)
    assert C.chain_ok(exp1, red1)                                    # stage-1 identity boundary
    assert C.chain_ok(exp1, conv(128, 256, 1))                       # stage-1 -> stage-2 entry
    assert not C.chain_ok(exp1, conv(64, 256, 3))                    # 3x3 next conv
    assert not C.chain_ok(conv(256, 64, 1, act="silu"), red1)        # non-ReLU epilogue
    assert C.chain_ok(conv(512, 128, 1), conv(128, 512, 1))         # stage 2 -> 128: conv_chain2
    assert not C.chain_ok(conv(512, 128, 1), conv(256, 512, 1))     # -> 256: removed (spilled)
    assert not C.chain_ok(conv(1024, 256, 1), conv(256, 1024, 1))   # stage 3: removed (slower)


def test_chain_dual_ok_requires_stride1_shortcut():
    conv = _resnet_specs()
    fused = C.fuse_shortcut(conv(256, 64, 1), conv(256, 64, 1))
    assert C.chain_dual_ok(fused, conv(64, 256, 1))
    assert not C.chain_dual_ok(fused, conv(128, 256, 1))
    strided = C.fuse_shortcut(conv(512, 128, 1), conv(512, 256, 1, stride=2))
    assert not C.chain_dual_ok(strided, conv(128, 512, 1))


def test_whisper_text_rendering_and_reply_filter():
    from aiko_services_amd.elements.gpu.speech import _reply
    from aiko_services_amd.models.whisper_decoder import EOT, SOT_SEQUENCE, attn_decode_work, decode_text
    rows = [list(SOT_SEQUENCE) + [10, 20, EOT, 30], list(SOT_SEQUENCE) + [EOT] * 3]
    assert decode_text(rows) == ["<10> <20>", ""]

    class Tok:
        def decode(self, ids):
            return " " + "".join(chr(97 + i % 26) for i in ids) + "."
    assert decode_text(rows, Tok()) == ["ku.", "."]
    assert _reply("") == "<silence>" and _reply("Thank you.") == "<silence>"
    assert _reply(" Hello World. ") == "hello world"
    assert attn_decode_work(16, 12, 1500) >= 16 * 12 * 66


def test_host_ring_never_reuses_a_held_result():
    """pinned result rings must not overwrite buffers a consumer still holds."""
    import gc
    from aiko_services_amd.gpu.element import DeviceResult, HostRing
    ring = HostRing(lambda: torch.zeros(4), initial=2, max_sets=6)
    held = []
    for k in range(5):                      # hold every result: the ring has to grow
        idx, buf = ring.acquire()
        buf.fill_(k)
        held.append(ring.bind(idx, DeviceResult({"x": buf}, None)))
    assert len(ring) == 5
    assert [int(r.tensors["x"][0]) for r in held] == [0, 1, 2, 3, 4]
    del held[:]
    gc.collect()
    for _ in range(10):                     # dropped results: sets are recycled, no growth
        idx, buf = ring.acquire()
        r = ring.bind(idx, DeviceResult({"x": buf}, None))
        del r
    assert len(ring) == 5
    keep = []
    for _ in range(6):
        idx, buf = ring.acquire()
        keep.append(ring.bind(idx, DeviceResult({"x": buf}, None)))
    import pytest
    with pytest.raises(RuntimeError):
        ring.acquire()


def test_hop_credits_hold_until_ack():
    """Forward hops hold a staging slot (a credit) until the response's ack; with every slot
    held the link refuses (NoCredit) instead of reusing a buffer a retransmit may need; a dead
    peer has no credit and keeps its held frames for re-dispatch."""
    import pytest
    from aiko_services_amd.parallel.hop import HopPlane, NoCredit
    plane = HopPlane([(0, 0)], device="cpu", depth=2)
    x = torch.arange(6.0)
    plane.encode(0, {"x": x}, key=("s", 0))
    plane.encode(0, {"x": x + 1}, key=("s", 1))
    assert plane.credit(0) == 0
    with pytest.raises(NoCredit):
        plane.encode(0, {"x": x}, key=("s", 2))
    assert torch.equal(plane.held_values(("s", 1))["x"], x + 1)     # the retransmit buffer
    plane.ack(("s", 0))
    assert plane.credit(0) == 1
    plane.encode(0, {"x": x + 2}, key=("s", 2))
    assert torch.equal(plane.held_values(("s", 1))["x"], x + 1)     # held slot never reused
    assert plane.stats()["held_frames"] == 2


def test_narrow_variant_eligibility():
    """The direct narrow-layer kernel (tuner variant 7) is offered exactly for 3x3 / pad 1 /
    stride 1-2 and 1x1 / stride 1 convs with 16 or 32 input and output channels."""
    g = torch.Generator().manual_seed(1)

    def conv(cout, cin, k, stride=1):
        return C.make_conv_spec(torch.randn(cout, cin, k, k, generator=g), None, stride=stride, pad=k // 2, act="silu")
    assert C.narrow_variant_ok(conv(16, 16, 3))
    assert C.narrow_variant_ok(conv(32, 16, 3, stride=2))
    assert C.narrow_variant_ok(conv(32, 32, 1))
    assert not C.narrow_variant_ok(conv(32, 32, 1, stride=2))          # 1x1 only at stride 1
    assert not C.narrow_variant_ok(conv(64, 32, 3))                    # Cout 64: buffer-DMA kernels
    assert not C.narrow_variant_ok(conv(32, 48, 3))                    # Cc 48
    assert not C.narrow_variant_ok(conv(32, 32, 5))                    # 5x5
    assert not C.narrow_variant_ok(conv(16, 16, 3), x2=torch.zeros(1))  # second source


def test_window_shift_cpu_path():
    """ops.audio.window_shift on host tensors: the AudioWindow update dst = src[:, n:] ++ chunk."""
    from aiko_services_amd.ops.audio import window_shift
    src = torch.arange(2 * 12, dtype=torch.float32).view(2, 12)
    chunk = -torch.arange(2 * 4, dtype=torch.float32).view(2, 4) - 1
    dst = torch.empty_like(src)
    window_shift(src, chunk, dst)
    assert torch.equal(dst, torch.cat([src[:, 4:], chunk], 1))


def test_native_library_has_every_kernel_stub():
    """Every kernel the launchers reference has its host stub in the built library (a target
    builtin reached by a __global__ template's host pass silently drops the stub, and the
    library then fails to load on the GPU box).  Skipped before the first build."""
    import os
    import shutil
    import subprocess
    import pytest
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "aiko_services_amd", "_C.so")
    nm = shutil.which("nm")
    if not os.path.exists(so) or nm is None:
        pytest.skip("native library not built here")
    out = subprocess.run([nm, "-D", "--undefined-only", so], capture_output=True, text=True).stdout
    missing = [line.split()[-1] for line in out.splitlines() if "device_stub" in line]
    assert not missing, missing[:5]
