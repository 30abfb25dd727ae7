"""Rank 0 of a 3-rank replicated-DP actor pipeline (``tensor_dp3_replicated.json`` on gloo) whose
rank-2 replica is SIGSTOPped mid-stream: alive, no last will, never posts its receives.
Driven by ``tests/test_hop_drop.py::test_stopped_replica``; prints one ``RESULT {json}`` line.

    python tests/native/stuck_replica.py DEFINITION.json

Phases: stream ``a`` runs until rank 2 is stopped and a frame held by it fails (ERROR after
``hop_timeout``); stream ``b`` must then complete on the other replicas while the stopped
peer's zero-copy send still holds its SyntheticFrames slot; rank 2 is resumed, the held slot
comes back, and stream ``c`` completes with rank 2 serving again."""
import json
import os
import queue
import signal
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(path):
    from aiko_services_amd.parallel.launch import create_rank_pipeline, join, spawn_workers, start_when_ready
    from aiko_services_amd.parallel.placement import make_plan
    from aiko_services_amd.runtime.actor import ActorTopic
    from aiko_services_amd.runtime.process import aiko
    with open(path) as f:
        plan = make_plan(json.load(f))
    manager, _ = spawn_workers(plan)
    plane = join(plan, 0)
    responses: queue.Queue = queue.Queue()
    pipeline = create_rank_pipeline(plan, 0, queue_response=responses, grace_time=600, auto_start=False)
    rank2 = manager.processes["rank2"]["process"].pid
    result = {}
    fid = [0]

    def stream(sid):
        pipeline._post_message(ActorTopic.IN, "create_stream", [sid, None, {"frames": 0}, 600, responses, None])
        while sid not in pipeline.stream_leases:
            time.sleep(0.01)

    def pool():
        node = pipeline.pipeline_graph.get_node("SyntheticFrames")
        return node.element.frame_pool

    def run(sid, n, stop_when=None, timeout=60.0):
        """n frames on ``sid`` (a window of 2 in flight); -> (ok, errors)."""
        stream(sid)
        ok, err, sent, done = 0, 0, 0, 0
        deadline = time.monotonic() + timeout
        while done < sent or (sent < n and err == 0):
            while sent < n and err == 0 and sent - done < 2:
                if not pipeline.admit_frame(sid, fid[0], timeout=0 if sent > done else 30):
                    break
                pipeline.create_frame({"stream_id": sid, "frame_id": fid[0]}, {})
                fid[0] += 1
                sent += 1
                if stop_when is not None:
                    stop_when(sent)
            try:
                info, _ = responses.get(timeout=max(0.1, deadline - time.monotonic()))
            except queue.Empty:
                break
            done += 1
            if info["state"] == 0:
                ok += 1
            else:
                err += 1
                break
        return ok, err

    def driver():
        try:
            t_stop = {}

            def stop(sent):
                if sent == 6 and not t_stop:
                    os.kill(rank2, signal.SIGSTOP)
                    t_stop["t"] = time.monotonic()
            ok_a, err_a = run("a", 200, stop_when=stop)
            result["a"] = [ok_a, err_a, round(time.monotonic() - t_stop.get("t", 0.0), 2)]
            time.sleep(0.5)                               # the timer has dropped every timed-out frame
            p = pool()
            result["stuck"] = {"dropped_pending": plane.stats()["dropped_pending"],
                               "suspect": plane.stats().get("suspect", []),
                               "pool_free": p.unheld_count(), "pool_slots": p.capacity}
            result["b"] = list(run("b", 12))
            result["stuck_after_b"] = {"dropped_pending": plane.stats()["dropped_pending"],
                                       "pool_free": pool().unheld_count(),
                                       "credit_to_2": plane.credit(2)}
            os.kill(rank2, signal.SIGCONT)
            deadline = time.monotonic() + 30
            # the slot comes back once the stuck send completes; the suspicion goes with the
            # first message from rank 2 (its late responses)
            while (plane.stats()["dropped_pending"] or pool().unheld_count() < pool().capacity
                   or plane.suspect) and time.monotonic() < deadline:
                time.sleep(0.05)
            result["resumed"] = {"dropped_pending": plane.stats()["dropped_pending"],
                                 "pool_free": pool().unheld_count(),
                                 "suspect": plane.stats().get("suspect", [])}
            seq2 = plane.send_links[2].seq
            result["c"] = list(run("c", 12))
            result["sent_to_2_in_c"] = plane.send_links[2].seq - seq2
            result["hop"] = {k: v for k, v in plane.stats().items() if not k.startswith("pool_free")}
        except Exception as exc:                          # noqa: BLE001
            result["error"] = repr(exc)
        finally:
            try:
                os.kill(rank2, signal.SIGCONT)
            except OSError:
                pass
            print("RESULT " + json.dumps(result), flush=True)
            aiko.process.terminate(0)

    start_when_ready(pipeline, then=lambda: threading.Thread(target=driver, daemon=True).start())
    pipeline.run(mqtt_connection_required=True)


if __name__ == "__main__":
    main(sys.argv[1])
