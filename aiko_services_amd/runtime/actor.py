"""Actors: Services with a control (priority) and an in mailbox (reference ``main/actor.py``).

An MQTT payload ``(method arg ...)`` on ``{actor}/in`` is parsed and posted to the actor's
``in`` mailbox; the event loop invokes ``method(*args)`` on the actor.  Local callers post
directly with ``_post_message(topic, command, args, delay=None, target_function=None)``;
``delay`` schedules through a timer.  Every actor owns an ECProducer over ``self.share``
(``lifecycle``, ``log_level``, ``running``) so its live variables are visible/editable
remotely (``log_level`` edits apply immediately).

Difference from the reference (Appendix A): a ``TypeError`` raised *inside* the target method
is logged, not turned into ``SystemExit``; only an arity mismatch of the call itself is
reported as an invocation error.
"""
from __future__ import annotations

import inspect
import os
import time
import traceback
from abc import abstractmethod

from ..utils.logger import DEBUG, get_log_level_name
from ..utils.sexpr import parse
from . import event
from .context import Interface
from .process import aiko
from .service import Service

__all__ = ["Actor", "ActorImpl", "ActorTest", "ActorTestImpl", "ActorTopic", "ActorMessage"]

_LOGGER = aiko.logger(__name__, log_level=os.environ.get("AIKO_LOG_LEVEL_ACTOR", "INFO"))


class ActorMessage:
    __slots__ = ("target_object", "command", "arguments", "target_function")

    def __init__(self, target_object, command, arguments, target_function=None):
        self.target_object = target_object
        self.command = command
        self.arguments = arguments
        self.target_function = target_function

    def __repr__(self):
        return f"Message: {self.command}({str(self.arguments)[1:-1]})"

    def invoke(self):
        if _LOGGER.isEnabledFor(DEBUG):
            _LOGGER.debug(f"Message.invoke(): {self}")
        fn = self.target_function
        if fn is None:
            fn = getattr(self.target_object, self.command, None)
        if fn is None:
            _LOGGER.error(f"{self}: Function not found in: {type(self.target_object).__name__}")
            return
        if not callable(fn):
            _LOGGER.error(f"{self}: isn't callable")
            return
        args = self.arguments
        if isinstance(args, dict):
            args = [args]
        try:
            fn(*args)
        except TypeError:
            # distinguish a bad call signature from a TypeError raised inside the method
            try:
                inspect.signature(fn).bind(*args)
                bind_ok = True
            except (TypeError, ValueError):
                bind_ok = False
            if bind_ok:
                _LOGGER.error(traceback.format_exc())
            else:
                _LOGGER.error(f"Message.invoke: {self.command} {self.arguments}: bad arguments")


# reference name
Message = ActorMessage


class ActorTopic:
    IN = "in"
    OUT = "out"
    CONTROL = "control"
    STATE = "state"
    topics = [CONTROL, STATE, IN, OUT]

    def __init__(self, topic_name):
        self.topic_name = topic_name


class Actor(Service):
    Interface.default("Actor", "aiko_services_amd.runtime.actor.ActorImpl")

    @abstractmethod
    def run(self, mqtt_connection_required=True):
        pass


class ActorImpl(Actor):
    @classmethod
    def proxy_post_message(cls, proxy_name, actual_object, actual_function, actual_function_name,
                           *args, **kwargs):
        """``ProxyAllMethods`` proxy function: calls become mailbox posts (control_* -> control)."""
        command = actual_function_name
        topic = ActorTopic.CONTROL if command.startswith(f"{ActorTopic.CONTROL}_") else ActorTopic.IN
        actual_object._post_message(topic, command, args, target_function=actual_function)

    def __init__(self, context):
        context.get_implementation("Service").__init__(self, context)
        if not hasattr(self, "logger"):
            self.logger = aiko.logger(context.name)
        self.share = {
            "lifecycle": "ready",
            "log_level": get_log_level_name(self.logger),
            "running": False,
        }
        from ..control.share import ECProducer
        self.ec_producer = ECProducer(self, self.share)
        self.ec_producer.add_handler(self.ec_producer_change_handler)
        self._delayed: list = []
        for topic in (ActorTopic.CONTROL, ActorTopic.IN):
            event.add_mailbox_handler(self._mailbox_handler, self._actor_mailbox_name(topic),
                                      priority=(topic == ActorTopic.CONTROL))
        self.add_message_handler(self._topic_in_handler, self.topic_in)

    def _actor_mailbox_name(self, topic):
        return f"{self.name}/{self.service_id}/{topic}"

    def _mailbox_handler(self, topic, message, time_posted):
        message.invoke()

    def _topic_in_handler(self, _aiko, topic, payload_in):
        command, parameters = parse(payload_in)
        self._post_message(ActorTopic.IN, command, parameters)

    def _post_message(self, topic, command, args, delay=None, target_function=None):
        message = ActorMessage(self, command, args, target_function=target_function)
        if not delay:
            event.mailbox_put(self._actor_mailbox_name(topic), message)
        else:
            self._delayed.append((time.time() + delay, topic, message))
            if len(self._delayed) == 1:
                event.add_timer_handler(self._post_delayed_message_handler, delay)

    def _post_delayed_message_handler(self):
        now = time.time()
        due = [d for d in self._delayed if d[0] <= now + 1e-3]
        self._delayed = [d for d in self._delayed if d[0] > now + 1e-3]
        for _, topic, message in due:
            event.mailbox_put(self._actor_mailbox_name(topic), message)
        event.remove_timer_handler(self._post_delayed_message_handler)
        if self._delayed:
            nxt = min(d[0] for d in self._delayed)
            event.add_timer_handler(self._post_delayed_message_handler, max(0.0, nxt - now))

    def __repr__(self):
        return f"[{type(self).__module__}.{type(self).__name__} object at {hex(id(self))}]"

    def ec_producer_change_handler(self, command, item_name, item_value):
        if item_name == "log_level":
            try:
                self.logger.setLevel(str(item_value).upper())
            except ValueError:
                pass

    def is_running(self):
        return self.share["running"]

    def run(self, mqtt_connection_required=True):
        self.share["running"] = True
        try:
            aiko.process.run(mqtt_connection_required=mqtt_connection_required)
        except Exception:
            _LOGGER.error(traceback.format_exc())
            raise
        finally:
            self.share["running"] = False

    def set_log_level(self, level):
        pass

    def stop(self):
        aiko.process.terminate()


class ActorTest(Actor):
    Interface.default("ActorTest", "aiko_services_amd.runtime.actor.ActorTestImpl")
    __test__ = False

    @abstractmethod
    def initialize(self):
        pass

    @abstractmethod
    def control_test(self, value):
        pass

    @abstractmethod
    def test(self, value):
        pass


class ActorTestImpl(ActorTest):
    """Mailbox-priority self test (reference ``actor.py:285-328``): records call order."""
    __test__ = False

    def __init__(self, context):
        context.get_implementation("Actor").__init__(self, context)
        self.test_count = None
        self.calls: list = []

    def initialize(self):
        self.control_test(0)
        self.test(1)
        self.test(2)
        self.control_test(3)
        self.test_count = 4

    def _mailbox_handler(self, topic, message, time_posted):
        ActorImpl._mailbox_handler(self, topic, message, time_posted)
        if topic == self._actor_mailbox_name(ActorTopic.IN):
            if self.test_count and self.test_count <= 5:
                self.control_test(self.test_count)
                self.test_count += 1

    def control_test(self, value):
        self.calls.append(("control_test", value))

    def test(self, value):
        self.calls.append(("test", value))
