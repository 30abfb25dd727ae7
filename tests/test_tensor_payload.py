"""Binary tensor payloads on the control plane (message/tensor_payload.py): arrays in a remote
call or a /out publication travel as one binary MQTT message, bit-exact; generate() refuses
them (never str(tensor)).  Reference: main/pipeline.py:1080-1090 (remote hop publishes the
element inputs), examples/xgo_robot/xgo_robot.py:320-324 (binary arrays over MQTT)."""
import numpy as np
import pytest
import torch

from aiko_services_amd.message import tensor_payload as tp
from aiko_services_amd.utils import sexpr
from aiko_services_amd.utils.sexpr import generate, parse


@pytest.mark.parametrize("native", [True, False])
def test_generate_refuses_arrays(native, monkeypatch):
    if not native:
        monkeypatch.setattr(sexpr, "_native", None)
    elif sexpr._native is None:
        pytest.skip("native S-expression module not built")
    for bad in (np.zeros(3), torch.zeros(2), torch.zeros((), dtype=torch.bfloat16)):
        with pytest.raises(TypeError):
            generate("process_frame", [{"stream_id": 1}, {"x": bad}])
    assert generate("a", [1, 2.5, True, None, "x y"]) == "(a 1 2.5 True 0: 3:x y)"


@pytest.mark.parametrize("codec", ["raw", "zlib"])
def test_roundtrip_dtypes_shapes(codec):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 3, 16, 16, generator=g)
    b = torch.randn(3, 5, generator=g).bfloat16()
    i8 = torch.randint(-128, 127, (7,), dtype=torch.int8, generator=g)
    nc = torch.randn(6, 4, generator=g).t()                      # non-contiguous
    u = np.arange(24, dtype=np.uint8).reshape(2, 3, 4)
    f16 = np.linspace(-2, 2, 9, dtype=np.float16)
    empty = torch.empty(0, 3)
    scalar = torch.tensor(3.25)
    params = [{"stream_id": "s", "frame_id": 3},
              {"x": x, "b": b, "i8": i8, "nc": nc, "u": u, "f16": f16, "empty": empty, "scalar": scalar,
               "nested": [b, "q", {"deep": u}], "n": 5, "none": None}]
    payload = tp.encode_message("process_frame", params, codec=codec)
    assert isinstance(payload, bytes) and tp.is_tensor_payload(payload)
    cmd, out = parse(payload)
    assert cmd == "process_frame" and out[0] == {"stream_id": "s", "frame_id": "3"}
    d = out[1]
    for k in ("x", "b", "i8", "nc", "empty", "scalar"):
        assert isinstance(d[k], torch.Tensor) and d[k].dtype == params[1][k].dtype
        assert torch.equal(d[k], params[1][k]), k
    assert d["u"].dtype == np.uint8 and np.array_equal(d["u"], u)
    assert d["f16"].dtype == np.float16 and np.array_equal(d["f16"], f16)
    assert torch.equal(d["nested"][0], b) and d["nested"][1] == "q" and np.array_equal(d["nested"][2]["deep"], u)
    assert d["n"] == "5" and d["none"] is None
    d["u"][0, 0, 0] = 99                                          # decoded arrays own their memory


def test_plain_messages_stay_text():
    assert tp.encode_message("add", ["a", 1, {"k": "v"}]) == "(add a 1 (k: v))"
    assert tp.encode_message("f", {"a": 1}) == generate("f", {"a": 1})
    payload = tp.encode_message("f", {"a": torch.ones(2)})      # dict parameters keep their keys
    cmd, params = parse(payload)
    assert cmd == "f" and torch.equal(params["a"], torch.ones(2))


def test_refuses_object_arrays_and_bad_blobs():
    with pytest.raises(TypeError):
        tp.encode_message("f", [np.array([object()], dtype=object)])
    payload = bytearray(tp.encode_message("f", [torch.ones(64)]))
    with pytest.raises(ValueError):
        tp.decode_message(bytes(payload[:-128]))                  # truncated: blob outside message


def test_device_result_travels_as_its_tensors():
    pytest.importorskip("aiko_services_amd.gpu.element")
    from aiko_services_amd.gpu.element import DeviceResult
    r = DeviceResult({"top_index": torch.arange(10).reshape(2, 5)}, None)
    with pytest.raises(TypeError):
        generate("f", [r])
    cmd, params = parse(tp.encode_message("f", [{"topk": r}]))
    got = params[0]["topk"]
    assert isinstance(got, DeviceResult) and torch.equal(got.wait()["top_index"], r.tensors["top_index"])


def test_process_keeps_tensor_payload_bytes():
    """The process router must not utf-8-decode a tensor payload on a text topic."""
    from aiko_services_amd.runtime.process import ProcessImplementation

    class M:
        topic = "ns/h/1/1/in"
        payload = tp.encode_message("process_frame", [{"stream_id": 1}, {"x": torch.arange(4.0)}])

    seen = []
    proc = ProcessImplementation()
    proc._message_handlers[M.topic] = [lambda _a, _t, p: seen.append(parse(p))]
    proc.on_message_queue_handler(M, "message")
    assert seen and torch.equal(seen[0][1][1]["x"], torch.arange(4.0))


def test_decode_refuses_inconsistent_or_inflated_blobs():
    """A header whose blob length or inflated size does not match the claimed array is refused
    (no allocation from the claim alone, no unbounded zlib inflation)."""
    import json
    import struct
    import zlib

    import numpy as np
    import pytest

    from aiko_services_amd.message.tensor_payload import MAGIC, decode_message, encode_message

    good = encode_message("f", [np.arange(12, dtype=np.int32)])
    decode_message(good)

    def forge(entry_patch, blob):
        hdr = {"v": 1, "sexpr": "(f 0:)", "results": [],
               "arrays": [dict({"path": [0], "kind": "numpy", "dtype": "<i4", "shape": [12], "device": "cpu",
                                "offset": 0, "nbytes": len(blob), "codec": "raw"}, **entry_patch)]}
        h = json.dumps(hdr).encode()
        lead = len(MAGIC) + 4 + len(h)
        return MAGIC + struct.pack("<I", len(h)) + h + b"\x00" * ((-lead) % 64) + blob

    with pytest.raises(ValueError):                       # 40 bytes for a 48-byte array
        decode_message(forge({}, b"\x01" * 40))
    with pytest.raises(ValueError):                       # absurd claimed shape
        decode_message(forge({"shape": [1 << 40, 1 << 20]}, b"\x01" * 48))
    bomb = zlib.compress(b"\x00" * (1 << 22))
    with pytest.raises(ValueError):                       # inflates past the 48 claimed bytes
        decode_message(forge({"codec": "zlib", "nbytes": len(bomb)}, bomb))
    with pytest.raises(ValueError):
        decode_message(forge({"shape": [-1]}, b"\x01" * 48))
