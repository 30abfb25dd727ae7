"""Configuration: AIKO_GPU_* environment settings."""
import pytest


def test_gpu_configuration_env(monkeypatch):
    """AIKO_GPU_* settings."""
    from aiko_services_amd.utils.configuration import get_gpu_configuration
    cfg = get_gpu_configuration()
    assert cfg.device is None and cfg.pp_depth == 2 and cfg.autotune and not cfg.graph
    assert cfg.device_for_local_rank(3) == 3
    monkeypatch.setenv("AIKO_GPU_DEVICE_MAP", "0,2,4,6")
    monkeypatch.setenv("AIKO_GPU_GRAPH", "true")
    monkeypatch.setenv("AIKO_GPU_PP_DEPTH", "4")
    monkeypatch.setenv("AIKO_GPU_COMM_TIMEOUT", "30")
    cfg = get_gpu_configuration()
    assert cfg.device_for_local_rank(1) == 2 and cfg.device_for_local_rank(5) == 2
    assert cfg.graph and cfg.pp_depth == 4 and cfg.comm_timeout_s == 30.0
    monkeypatch.setenv("AIKO_GPU_DEVICE", "7")
    assert get_gpu_configuration().device_for_local_rank(1) == 7
    monkeypatch.setenv("AIKO_GPU_MEMORY_FRACTION", "1.5")
    with pytest.raises(ValueError):
        get_gpu_configuration()
