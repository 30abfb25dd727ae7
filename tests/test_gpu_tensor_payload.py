"""GPU world-1 variant of the plain-remote tensor round trip: a DEVICE tensor crosses a
``deploy.remote`` hop with no RCCL plan (binary MQTT payload, host-staged) and comes back on
the GPU bit-exact; the child receives it on its GPU."""
import pytest

pytestmark = pytest.mark.gpu


def test_device_tensor_through_plain_remote():
    from aiko_services_amd.tools.tensor_echo import orchestrate
    res = orchestrate(frames=3, device="cuda", timeout=90)
    assert "error" not in res, res
    assert res["frames"] == 3 and res["mismatches"] == [], res
    assert str(res["device_in"]).startswith("cuda"), res
