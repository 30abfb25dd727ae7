"""Example / test PipelineElements referenced by the example PipelineDefinitions
(reference ``examples/pipeline/elements.py:49-324``): PE_Add, PE_Inspect, PE_Metrics,
PE_RandomIntegers, PE_0..PE_4, PE_IN/PE_TEXT/PE_OUT, PE_DataDecode/PE_DataEncode.
"""
from __future__ import annotations

import base64
import random
import time
from io import BytesIO

import numpy as np

from aiko_services_amd.pipeline.engine import PipelineElement
from aiko_services_amd.pipeline.stream import StreamEvent
from aiko_services_amd.utils.sexpr import parse

__all__ = ["PE_Add", "PE_Inspect", "PE_Metrics", "PE_RandomIntegers", "PE_0", "PE_1", "PE_2",
           "PE_3", "PE_4", "PE_IN", "PE_TEXT", "PE_OUT", "PE_DataDecode", "PE_DataEncode"]


def _all_outputs(element, stream):
    frame = stream.frames[stream.frame_id]
    return {o["name"]: frame.swag[o["name"]] for o in element.definition.output if o["name"] in frame.swag}


class _PE(PipelineElement):
    PROTOCOL = None

    def __init__(self, context):
        if self.PROTOCOL:
            context.set_protocol(self.PROTOCOL)
        context.get_implementation("PipelineElement").__init__(self, context)


class PE_Add(_PE):
    PROTOCOL = "add:0"

    def process_frame(self, stream, i):
        constant, _ = self.get_parameter("constant", default=1)
        i_new = int(i) + int(constant)
        self.logger.debug(f"{self.my_id()} i in: {i}, out: {i_new}")
        delay, _ = self.get_parameter("delay", default=0)
        if delay:
            time.sleep(float(delay))
        return StreamEvent.OKAY, {"i": i_new}


class PE_Inspect(_PE):
    PROTOCOL = "inspect:0"

    def _inspect_file(self, stream, target):
        f = stream.variables.get("inspect_file")
        if f is None:
            f = open(target.split(":", 1)[1], "a")
            stream.variables["inspect_file"] = f
        return f

    def process_frame(self, stream):
        frame = stream.frames[stream.frame_id]
        enable, _ = self.get_parameter("enable", True)
        if str(enable).lower() not in ("false", "0"):
            names, found = self.get_parameter("inspect")
            if found:
                head, rest = parse(str(names))
                names = [head] + list(rest)
                if "*" in names:
                    names = list(frame.swag.keys())
            else:
                names = list(frame.swag.keys())
            target, _ = self.get_parameter("target", "log")
            f = self._inspect_file(stream, target) if target.startswith("file:") else None
            for name in names:
                line = f"{self.my_id()} {name}: {frame.swag.get(name)}"
                if f is not None:
                    f.write(line + "\n")
                elif target == "log":
                    self.logger.info(line)
                elif target == "print":
                    print(line)
                else:
                    return StreamEvent.ERROR, {"diagnostic": "'target' parameter must be 'file', 'log' or 'print'"}
            if f is not None:
                f.flush()
        return StreamEvent.OKAY, _all_outputs(self, stream)

    def stop_stream(self, stream, stream_id):
        f = stream.variables.pop("inspect_file", None)
        if f is not None:
            f.close()
        return StreamEvent.OKAY, {}


class PE_Metrics(_PE):
    PROTOCOL = "metrics:0"

    def process_frame(self, stream):
        metrics = stream.frames[stream.frame_id].metrics
        for name, value in metrics.get("pipeline_elements", {}).items():
            self.logger.debug(f"{name}: {value * 1000:.3f} ms")
        self.logger.debug(f"Pipeline total: {metrics.get('time_pipeline', 0.0) * 1000:.3f} ms")
        return StreamEvent.OKAY, _all_outputs(self, stream)


class PE_RandomIntegers(_PE):
    PROTOCOL = "random_integers:0"

    def __init__(self, context):
        super().__init__(context)
        self.share["random"] = "?"

    def start_stream(self, stream, stream_id):
        rate, _ = self.get_parameter("rate", default=1.0)
        self.create_frames(stream, self.frame_generator, rate=float(rate))
        return StreamEvent.OKAY, {}

    def frame_generator(self, stream, frame_id):
        limit, _ = self.get_parameter("limit")
        if frame_id < int(limit):
            return StreamEvent.OKAY, {"random": random.randint(0, 9)}
        return StreamEvent.STOP, {"diagnostic": "Frame limit reached"}

    def process_frame(self, stream, random):
        self.ec_producer.update("random", random)
        return StreamEvent.OKAY, {"random": random}


class PE_0(_PE):
    PROTOCOL = "increment:0"

    def process_frame(self, stream, a):
        inc, _ = self.get_parameter("pe_0_inc", 1)
        return StreamEvent.OKAY, {"b": int(a) + int(inc)}


class PE_1(_PE):
    PROTOCOL = "increment:0"

    def process_frame(self, stream, b):
        inc, _ = self.get_parameter("pe_1_inc", 1)
        return StreamEvent.OKAY, {"c": int(b) + int(inc)}


class PE_2(_PE):
    PROTOCOL = "increment:0"

    def process_frame(self, stream, c):
        return StreamEvent.OKAY, {"d": int(c) + 1}


class PE_3(_PE):
    PROTOCOL = "increment:0"

    def process_frame(self, stream, c):
        return StreamEvent.OKAY, {"e": int(c) + 1}


class PE_4(_PE):
    PROTOCOL = "sum:0"

    def process_frame(self, stream, d, e):
        return StreamEvent.OKAY, {"f": int(d) + int(e)}


class PE_IN(_PE):
    PROTOCOL = "in:0"

    def process_frame(self, stream, in_a):
        return StreamEvent.OKAY, {"text_b": f"{in_a}:in"}


class PE_TEXT(_PE):
    PROTOCOL = "text_to_text:0"

    def process_frame(self, stream, text_b):
        return StreamEvent.OKAY, {"text_b": f"{text_b}:text"}


class PE_OUT(_PE):
    PROTOCOL = "out:0"

    def process_frame(self, stream, text_b):
        return StreamEvent.OKAY, {"out_c": f"{text_b}:out"}


class PE_DataDecode(_PE):
    """base64(np.save(array)) -> array (numeric arrays only: pickles are refused)."""

    def process_frame(self, stream, data):
        raw = base64.b64decode(data.encode("utf-8") if isinstance(data, str) else data)
        return StreamEvent.OKAY, {"data": np.load(BytesIO(raw), allow_pickle=False)}


class PE_DataEncode(_PE):
    def process_frame(self, stream, data):
        if isinstance(data, str):
            data = data.encode()
        if isinstance(data, np.ndarray):
            buf = BytesIO()
            np.save(buf, data, allow_pickle=False)
            data = buf.getvalue()
        return StreamEvent.OKAY, {"data": base64.b64encode(data).decode("utf-8")}
