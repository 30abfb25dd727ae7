"""Event engine, composition, actors, leases, EC share and the in-process control plane."""
import queue
import threading
import time
from abc import abstractmethod

import pytest

from aiko_services_amd.runtime import event
from aiko_services_amd.runtime.event import EventEngine


# ---- event engine (own instance, virtual clock) ---------------------------------------------

class FakeClock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def test_timers_heap_virtual_clock():
    clock = FakeClock()
    eng = EventEngine(clock=clock)
    calls = []
    eng.add_timer_handler(lambda: calls.append("a"), 1.0)
    eng.add_timer_handler(lambda: calls.append("b"), 0.5)
    eng.run_once()
    assert calls == []
    clock.t += 0.6
    eng.run_once()
    assert calls == ["b"]
    clock.t += 0.5
    eng.run_once()
    assert sorted(calls) == ["a", "b", "b"]


def test_timer_remove_and_immediate():
    clock = FakeClock()
    eng = EventEngine(clock=clock)
    calls = []

    def h():
        calls.append(1)
    eng.add_timer_handler(h, 1.0, immediate=True)
    eng.run_once()
    assert calls == [1]
    assert eng.remove_timer_handler(h)
    assert not eng.remove_timer_handler(h)
    clock.t += 5
    eng.run_once()
    assert calls == [1]


def test_mailbox_priority_and_queue():
    eng = EventEngine()
    order = []
    eng.add_mailbox_handler(lambda n, item, t: order.append(("in", item)), "a/1/in")
    eng.add_mailbox_handler(lambda n, item, t: order.append(("ctl", item)), "a/1/control")
    eng.add_queue_handler(lambda item, typ: order.append(("q", item)), ["message"])
    eng.mailbox_put("a/1/in", 1)
    eng.mailbox_put("a/1/in", 2)
    eng.mailbox_put("a/1/control", 3)
    eng.queue_put("m", "message")
    eng.run_once()
    assert order[0] == ("q", "m")
    assert order[1] == ("ctl", 3)          # priority mailbox drained before "in"
    assert order[2:] == [("in", 1), ("in", 2)]


def test_loop_wakeup_latency_and_throughput():
    """Wakeup-driven loop: thousands of queued messages per second (reference: ~100/s)."""
    eng = EventEngine()
    got = []
    done = threading.Event()
    n = 20000

    def handler(item, typ):
        got.append(item)
        if len(got) == n:
            done.set()
    eng.add_queue_handler(handler, ["message"])
    t = threading.Thread(target=eng.loop, args=(True,), daemon=True)
    t.start()
    t0 = time.perf_counter()
    for i in range(n):
        eng.queue_put(i, "message")
    assert done.wait(10)
    rate = n / (time.perf_counter() - t0)
    eng.terminate()
    t.join(2)
    assert got == list(range(n))
    assert rate > 5000, rate


def test_call_soon_runs_on_loop_thread():
    eng = EventEngine()
    t = threading.Thread(target=eng.loop, args=(True,), daemon=True)
    t.start()
    fut = eng.call_soon(lambda: threading.current_thread().name)
    assert fut.result(5) == t.name
    eng.terminate()
    t.join(2)


# ---- composition --------------------------------------------------------------------------

def test_compose_frankenstein_class():
    from aiko_services_amd.runtime.context import Interface, compose_class, compose_instance, service_args

    class Greeter(Interface):
        Interface.default("Greeter", "tests.test_runtime_helpers.GreeterImpl")

        @abstractmethod
        def greet(self, name):
            pass

    class MyGreeterImpl(Greeter):
        def __init__(self, context):
            self.context = context

        def greet(self, name):
            return f"hi {name}"

    cls, impls = compose_class(MyGreeterImpl)
    assert "Greeter" in impls
    obj = compose_instance(MyGreeterImpl, service_args("g"))
    assert obj.greet("x") == "hi x"

    class Missing(Interface):
        @abstractmethod
        def f(self):
            pass

    class Bad(Missing):
        def __init__(self, context):
            pass
    with pytest.raises(ValueError):
        compose_class(Bad)


# ---- in-process process singleton on a Loopback bus ------------------------------------------

@pytest.fixture(scope="module")
def aiko_process():
    import aiko_services_amd as aiko
    from aiko_services_amd.message import Loopback, LoopbackBus
    if not aiko.process.initialized:
        aiko.process.run_in_thread(loop_when_no_handlers=True, message=Loopback(bus=LoopbackBus()))
    deadline = time.time() + 5
    while not event.is_running() and time.time() < deadline:
        time.sleep(0.01)
    return aiko


def test_actor_remote_call_and_mailbox(aiko_process):
    aiko = aiko_process
    from aiko_services_amd.runtime.actor import Actor
    from aiko_services_amd.runtime.context import Interface, actor_args, compose_instance

    results = queue.Queue()

    class Echo(Actor):
        @abstractmethod
        def echo(self, value):
            pass

    class EchoImpl(Echo):
        def __init__(self, context):
            context.get_implementation("Actor").__init__(self, context)

        def echo(self, value, extra=None):
            results.put((value, extra, threading.current_thread() is event.engine.loop_thread))

    Interface.default("Echo", EchoImpl)
    actor = event.call_on_loop(lambda: compose_instance(EchoImpl, actor_args("echo")))
    # remote-style call: S-expression on the actor's /in topic
    aiko.aiko.message.publish(actor.topic_in, "(echo hello)")
    v, extra, on_loop = results.get(timeout=5)
    assert v == "hello" and extra is None and on_loop
    proxy = aiko.get_actor_mqtt(actor.topic_in, Echo)
    proxy.echo("world")
    assert results.get(timeout=5)[0] == "world"
    actor._post_message("in", "echo", ["local", "x"])
    assert results.get(timeout=5)[:2] == ("local", "x")
    # delayed post
    t0 = time.time()
    actor._post_message("in", "echo", ["late"], delay=0.2)
    assert results.get(timeout=5)[0] == "late" and time.time() - t0 >= 0.18


def test_actor_mailbox_priority_selftest(aiko_process):
    from aiko_services_amd.runtime.actor import ActorTestImpl
    from aiko_services_amd.runtime.context import actor_args, compose_instance
    from aiko_services_amd.runtime.proxy import ProxyAllMethods

    def build():
        a = compose_instance(ActorTestImpl, actor_args("actor_test"))
        from aiko_services_amd.runtime.actor import ActorImpl
        p = ProxyAllMethods("actor_test", a, ActorImpl.proxy_post_message)
        return a, p
    actor, proxy = event.call_on_loop(build)
    proxy.initialize()
    deadline = time.time() + 5
    while len(actor.calls) < 6 and time.time() < deadline:
        time.sleep(0.01)
    # control_* calls go through the priority mailbox
    assert ("control_test", 0) in actor.calls and ("test", 1) in actor.calls


def test_lease_expiry_and_extend(aiko_process):
    from aiko_services_amd.runtime.lease import Lease
    expired = queue.Queue()
    lease = event.call_on_loop(lambda: Lease(0.2, "L1", lease_expired_handler=expired.put))
    time.sleep(0.1)
    event.call_on_loop(lease.extend)
    time.sleep(0.15)
    assert expired.empty()
    assert expired.get(timeout=2) == "L1"
    extended = queue.Queue()
    lease2 = event.call_on_loop(lambda: Lease(0.3, "L2", lease_extend_handler=lambda t, u: extended.put(u),
                                              automatic_extend=True))
    assert extended.get(timeout=2) == "L2"
    event.call_on_loop(lease2.terminate)


def test_ec_share_producer_consumer(aiko_process):
    aiko = aiko_process
    from aiko_services_amd.control.share import ECConsumer, ECProducer
    from aiko_services_amd.runtime.connection import ConnectionState
    from aiko_services_amd.runtime.context import compose_instance, service_args
    from aiko_services_amd.runtime.service import ServiceImpl

    changes = queue.Queue()

    def build():
        producer_service = compose_instance(ServiceImpl, service_args("ec_producer"))
        share = {"lifecycle": "ready", "nested": {"a": 1, "b": "two words"}}
        producer = ECProducer(producer_service, share)
        consumer_service = compose_instance(ServiceImpl, service_args("ec_consumer"))
        cache = {}
        consumer = ECConsumer(consumer_service, 0, cache, producer_service.topic_control, "*")
        consumer.add_handler(lambda cid, cmd, name, value: changes.put((cmd, name, value)))
        # pretend a registrar is present so the consumer requests the share
        aiko.aiko.connection.update_state(ConnectionState.REGISTRAR)
        return producer, consumer, cache
    producer, consumer, cache = event.call_on_loop(build)
    deadline = time.time() + 5
    while consumer.cache_state != "ready" and time.time() < deadline:
        time.sleep(0.01)
    assert consumer.cache_state == "ready"
    assert cache["nested"]["b"] == "two words"
    event.call_on_loop(lambda: producer.update("nested.a", 5))
    deadline = time.time() + 5
    while cache["nested"]["a"] != "5" and time.time() < deadline:
        time.sleep(0.01)
    assert cache["nested"]["a"] == "5"
    # remote edit on /control (how the dashboard edits variables)
    aiko.aiko.message.publish(producer.topic_in, "(update lifecycle busy)")
    deadline = time.time() + 5
    while producer.share["lifecycle"] != "busy" and time.time() < deadline:
        time.sleep(0.01)
    assert producer.share["lifecycle"] == "busy"
    event.call_on_loop(lambda: producer.remove("nested.b"))
    deadline = time.time() + 5
    while "b" in cache["nested"] and time.time() < deadline:
        time.sleep(0.01)
    assert "b" not in cache["nested"]
    event.call_on_loop(consumer.terminate)
    from aiko_services_amd.runtime.connection import ConnectionState as CS
    event.call_on_loop(lambda: aiko.aiko.connection.update_state(CS.TRANSPORT))


def test_xgo_robot_simulated_video_and_control(aiko_process):
    """examples/xgo_robot: simulated robot actor publishes zlib(np.save) frames on a binary topic,
    the controller decodes them and drives the robot through an XGORobot remote proxy."""
    from aiko_services_amd.examples.xgo_robot.robot_control import RobotControlImpl
    from aiko_services_amd.examples.xgo_robot.xgo_robot import XGORobotImpl, decode_image, encode_image
    from aiko_services_amd.runtime.context import actor_args, compose_instance
    import numpy as np
    img = np.arange(24, dtype=np.uint8).reshape(2, 4, 3)
    assert np.array_equal(decode_image(encode_image(img)), img)

    def make():
        ra = actor_args("xgo_robot")
        ra.update(fps=50.0, width=32, height=24)
        robot = compose_instance(XGORobotImpl, ra)
        ca = actor_args("robot_control")
        ca.update(robot_topic=robot.topic_in)
        return robot, compose_instance(RobotControlImpl, ca)
    robot, control = event.call_on_loop(make)
    deadline = time.time() + 5
    while int(control.share["frames_received"]) < 5 and time.time() < deadline:
        time.sleep(0.02)
    assert int(control.share["frames_received"]) >= 5
    assert control.last_image.shape == (24, 32, 3)
    control.robot("move", "x", 10)
    control.robot("turn", 500)          # clipped to 100 deg/s
    control.robot("claw", 128)
    deadline = time.time() + 5
    while (robot.share["pose"][0] == 0 or robot.share["claw"] != 128) and time.time() < deadline:
        time.sleep(0.02)
    assert robot.share["claw"] == 128 and robot._turn_rate == 100.0
    assert robot.share["pose"][0] != 0 or robot.share["pose"][1] != 0
    control.robot("stop")
    event.call_on_loop(lambda: event.remove_timer_handler(robot._tick))
    # VideoTest: the controller also consumes the test video source; live sleep_period retune
    from aiko_services_amd.examples.xgo_robot.robot_control import VideoTestImpl
    vt = event.call_on_loop(lambda: compose_instance(VideoTestImpl, actor_args("video_test")))
    start = int(control.share["frames_received"])
    event.call_on_loop(lambda: vt.ec_producer.update("sleep_period", 0.01))
    deadline = time.time() + 5
    while int(control.share["frames_received"]) < start + 5 and time.time() < deadline:
        time.sleep(0.02)
    assert int(control.share["frames_received"]) >= start + 5
    assert control.last_image.shape == (240, 320, 3) and vt._period == 0.01
    event.call_on_loop(lambda: event.remove_timer_handler(vt._tick))


def test_ec_test_services(aiko_process):
    """tools/ec_test: ECConsumerTest mirrors ECProducerTest's share and sees live log_level edits."""
    aiko = aiko_process
    from aiko_services_amd.control.share import PROTOCOL_EC_CONSUMER, PROTOCOL_EC_PRODUCER
    from aiko_services_amd.runtime.connection import ConnectionState
    from aiko_services_amd.runtime.context import compose_instance, service_args
    from aiko_services_amd.tools.ec_test import ECConsumerTest, ECProducerTest

    def build():
        p = compose_instance(ECProducerTest, service_args("ec_producer_test", protocol=PROTOCOL_EC_PRODUCER,
                                                          tags=["ec=true"]))
        args = service_args("ec_consumer_test", protocol=PROTOCOL_EC_CONSUMER, tags=["ec=true"])
        args.update(ec_producer_pid="0", ec_producer_topic_control=p.topic_control)
        c = compose_instance(ECConsumerTest, args)
        aiko.aiko.connection.update_state(ConnectionState.REGISTRAR)
        return p, c
    producer, consumer = event.call_on_loop(build)
    deadline = time.time() + 5
    while consumer.ec_consumer.cache_state != "ready" and time.time() < deadline:
        time.sleep(0.01)
    assert consumer.share_consumer["items"]["key_1"] == ["item_1a", "item_1b"]
    aiko.aiko.message.publish(producer.topic_control, "(update log_level DEBUG)")
    deadline = time.time() + 5
    while consumer.share_consumer.get("log_level") != "DEBUG" and time.time() < deadline:
        time.sleep(0.01)
    assert consumer.share_consumer["log_level"] == "DEBUG"
    assert ("update", "log_level", "DEBUG") in producer.changes
    event.call_on_loop(consumer.ec_consumer.terminate)
    event.call_on_loop(lambda: aiko.aiko.connection.update_state(ConnectionState.TRANSPORT))


def test_mailbox_stress_many_producers():
    """mailboxes and the queue under concurrent producers — every item delivered
    exactly once, per-producer FIFO order kept, priority mailbox never starved."""
    eng = EventEngine()
    producers, per = 8, 3000
    got_in, got_ctl, got_q = [], [], []
    eng.add_mailbox_handler(lambda n, item, t: got_ctl.append(item), "s/1/control")
    eng.add_mailbox_handler(lambda n, item, t: got_in.append(item), "s/1/in")
    eng.add_queue_handler(lambda item, typ: got_q.append(item), ["message"])
    t = threading.Thread(target=eng.loop, kwargs={"loop_when_no_handlers": True}, daemon=True)
    t.start()

    def produce(p):
        for i in range(per):
            eng.mailbox_put("s/1/in", (p, i))
            if i % 10 == 0:
                eng.mailbox_put("s/1/control", (p, i))
            if i % 7 == 0:
                eng.queue_put((p, i), "message")
    ths = [threading.Thread(target=produce, args=(p,)) for p in range(producers)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    deadline = time.time() + 20
    while (len(got_in) < producers * per or len(got_ctl) < producers * per // 10) and time.time() < deadline:
        time.sleep(0.01)
    eng.terminate()
    t.join(5)
    assert len(got_in) == producers * per and len(set(got_in)) == producers * per
    assert len(got_ctl) == producers * (per // 10)
    assert len(got_q) == producers * len(range(0, per, 7))
    for p in range(producers):
        seq = [i for (q, i) in got_in if q == p]
        assert seq == sorted(seq)                 # per-producer FIFO
