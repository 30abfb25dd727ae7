"""L1 message transports (control plane): MQTT (own client + broker), Castaway, Loopback."""
from .message import MQTT, Castaway, Loopback, LoopbackBus, Message  # noqa: F401
from .mqtt_broker import Broker, start_broker_thread  # noqa: F401
from .mqtt_client import MQTTClient, MQTTMessage  # noqa: F401
