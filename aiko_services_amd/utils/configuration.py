"""Environment-driven configuration (reference ``utilities/configuration.py``).

Same environment contract: ``AIKO_NAMESPACE``, ``AIKO_MQTT_HOST``, ``AIKO_MQTT_PORT``,
``AIKO_MQTT_TRANSPORT``, ``AIKO_MQTT_TLS``, ``AIKO_USERNAME``, ``AIKO_PASSWORD``.  The broker is
found by probing a TCP connect over (env host, localhost).  Additional MI355X knobs:
``AIKO_GPU_DEVICE`` (device index for this process), ``AIKO_GPU_FRAME_POOL_MB``.

The UDP bootstrap responder is implemented (and fixed: the reference's never ran) but only
started on request (:func:`bootstrap_start`).
"""
from __future__ import annotations

import getpass
from dataclasses import dataclass
import os
import secrets
import socket
import threading

__all__ = [
    "create_password", "get_hostname", "get_mqtt_configuration", "get_mqtt_host",
    "get_mqtt_port", "get_namespace", "get_namespace_prefix", "get_pid", "get_username",
    "bootstrap_start", "get_lan_ip_address", "GpuConfiguration", "get_gpu_configuration",
]

AIKO_BOOTSTRAP_UDP_PORT = 4149
AIKO_MQTT_HOSTS: list = []  # extra (host, port) candidates
AIKO_MQTT_HOST = "localhost"
AIKO_MQTT_PORT = 1883
AIKO_MQTT_TRANSPORT = "tcp"
AIKO_NAMESPACE = "aiko"
LOCALHOST_IP = "127.0.0.1"


def create_password(length: int = 32) -> str:
    return secrets.token_hex(length)


def get_lan_ip_address() -> str:
    try:
        ips = [ip for ip in socket.gethostbyname_ex(socket.gethostname())[2]
               if not ip.startswith("127.")]
        return ips[0] if ips else LOCALHOST_IP
    except Exception:
        return LOCALHOST_IP


def _host_server_up(host: str, port: int, timeout: float = 0.5) -> bool:
    try:
        with socket.create_connection((host, port), timeout=timeout):
            return True
    except OSError:
        return False


_hostname_cache: str | None = None


def get_hostname() -> str:
    global _hostname_cache
    if _hostname_cache is None:
        hostname = socket.gethostname()
        if "." not in hostname and hostname == "localhost":
            try:
                hostname = socket.gethostbyaddr(hostname)[0]
            except OSError:
                pass
        if hostname.endswith("amazonaws.com"):  # shorten AWS EC2 hostnames
            hyphen = hostname.find("-") + 1
            fullstop = hostname.find(".")
            hostname = hostname[hyphen:fullstop].replace("-", ".")
        _hostname_cache = hostname
    return _hostname_cache


def get_mqtt_port() -> int:
    return int(os.environ.get("AIKO_MQTT_PORT", AIKO_MQTT_PORT))


def get_mqtt_host():
    """Probe candidate brokers in order; returns (server_up, host, port)."""
    hosts = list(AIKO_MQTT_HOSTS)
    port = get_mqtt_port()
    env_host = os.environ.get("AIKO_MQTT_HOST")
    if env_host:
        hosts.insert(0, (env_host, port))
    hosts.append((AIKO_MQTT_HOST, port))
    for h, p in hosts:
        if _host_server_up(h, p):
            return True, h, p
    return False, env_host or AIKO_MQTT_HOST, port


def get_mqtt_configuration(tls_enabled=None):
    server_up, host, port = get_mqtt_host()
    transport = os.environ.get("AIKO_MQTT_TRANSPORT", AIKO_MQTT_TRANSPORT)
    username = os.environ.get("AIKO_USERNAME")
    password = os.environ.get("AIKO_PASSWORD")
    if tls_enabled is None:
        tls = os.environ.get("AIKO_MQTT_TLS")
        tls_enabled = (tls == "true") if tls else bool(username)
    return server_up, host, port, transport, username, password, tls_enabled


def get_namespace() -> str:
    return os.environ.get("AIKO_NAMESPACE", AIKO_NAMESPACE)


def get_namespace_prefix() -> str:
    ns = get_namespace()
    return ns[:ns.find(":") + 1] if ":" in ns else ""


def get_pid() -> str:
    return str(os.getpid())


def get_username() -> str:
    try:
        return getpass.getuser()
    except Exception:
        return "unknown"


# ---- UDP bootstrap: "boot? ip port" -> "boot mqtt_ip mqtt_port namespace" ----------------

def _bootstrap_loop(sock: socket.socket):
    response = f"boot {get_lan_ip_address()} {get_mqtt_port()} {get_namespace()}".encode()
    while True:
        try:
            message, _ = sock.recvfrom(256)
        except OSError:
            return
        tokens = message.decode("utf-8", "replace").split()
        if len(tokens) == 3 and tokens[0] == "boot?":
            try:
                sock.sendto(response, (tokens[1], int(tokens[2])))
            except (OSError, ValueError):
                pass


def bootstrap_start(port: int = AIKO_BOOTSTRAP_UDP_PORT) -> socket.socket:
    sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.bind(("0.0.0.0", port))
    threading.Thread(target=_bootstrap_loop, args=(sock,), daemon=True).start()
    return sock


# ---- GPU data-plane settings (AIKO_GPU_*; SURVEY §5.6 "add AIKO_GPU_*") ------------------

@dataclass(frozen=True)
class GpuConfiguration:
    """Process-wide defaults for the GPU data plane; element / definition parameters override.

    ========================  =========================================================  =======
    variable                  meaning                                                    default
    ========================  =========================================================  =======
    AIKO_GPU_DEVICE           device index of this process (else LOCAL_RANK)             LOCAL_RANK
    AIKO_GPU_DEVICE_MAP       comma list: local rank -> device index ("0,2,4,6")         identity
    AIKO_GPU_MEMORY_FRACTION  cap on this process's share of HBM (0 < f <= 1)            1.0
    AIKO_GPU_GRAPH            capture GPU elements into hipGraphs by default             false
    AIKO_GPU_AUTOTUNE         measure kernel tiles / variants on first use               true
    AIKO_GPU_TIMING           HIP-event timing per element into frame.metrics            false
    AIKO_GPU_PP_DEPTH         pipeline-parallel slot-ring depth per stage link           2
    AIKO_GPU_COMM_BACKEND     torch.distributed backend (nccl = RCCL on ROCm, or gloo)   auto
    AIKO_GPU_COMM_TIMEOUT     collective / P2P timeout in seconds                        600
    ========================  =========================================================  =======
    """
    device: int | None = None
    device_map: tuple = ()
    memory_fraction: float = 1.0
    graph: bool = False
    autotune: bool = True
    timing: bool = False
    pp_depth: int = 2
    comm_backend: str | None = None
    comm_timeout_s: float = 600.0

    def device_for_local_rank(self, local_rank: int) -> int:
        if self.device is not None:
            return self.device
        if self.device_map:
            return self.device_map[local_rank % len(self.device_map)]
        return local_rank


def _env_bool(name: str, default: bool) -> bool:
    v = os.environ.get(name)
    return default if v is None else v.strip().lower() in ("1", "true", "yes", "on")


def get_gpu_configuration() -> GpuConfiguration:
    dev = os.environ.get("AIKO_GPU_DEVICE")
    dmap = os.environ.get("AIKO_GPU_DEVICE_MAP", "")
    frac = float(os.environ.get("AIKO_GPU_MEMORY_FRACTION", "1.0"))
    if not 0.0 < frac <= 1.0:
        raise ValueError(f"AIKO_GPU_MEMORY_FRACTION must be in (0, 1], not {frac}")
    return GpuConfiguration(
        device=int(dev) if dev not in (None, "") else None,
        device_map=tuple(int(x) for x in dmap.split(",") if x.strip()),
        memory_fraction=frac,
        graph=_env_bool("AIKO_GPU_GRAPH", False),
        autotune=_env_bool("AIKO_GPU_AUTOTUNE", True),
        timing=_env_bool("AIKO_GPU_TIMING", False),
        pp_depth=int(os.environ.get("AIKO_GPU_PP_DEPTH", "2")),
        comm_backend=os.environ.get("AIKO_GPU_COMM_BACKEND") or None,
        comm_timeout_s=float(os.environ.get("AIKO_GPU_COMM_TIMEOUT", "600")))
