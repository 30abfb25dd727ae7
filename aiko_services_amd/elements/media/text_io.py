"""Text elements (reference ``elements/media/text_io.py:64-179``)."""
from __future__ import annotations

from pathlib import Path

from ...pipeline.engine import PipelineElement
from ...pipeline.stream import StreamEvent
from .common_io import DataSource, DataTarget

__all__ = ["TextOutput", "TextReadFile", "TextSample", "TextTransform", "TextWriteFile"]


class TextOutput(PipelineElement):
    def __init__(self, context):
        context.set_protocol("text_output:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, texts):
        return StreamEvent.OKAY, {"texts": texts}


class TextReadFile(DataSource):
    def __init__(self, context):
        context.set_protocol("text_read_file:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, paths):
        texts = []
        for path in paths:
            try:
                texts.append(Path(path).read_text())
            except Exception as exc:
                return StreamEvent.ERROR, {"diagnostic": f"Error loading text: {exc}"}
        return StreamEvent.OKAY, {"texts": texts}


class TextSample(PipelineElement):
    """Pass every ``sample_rate``-th frame, DROP_FRAME the others."""

    def __init__(self, context):
        context.set_protocol("text_sample:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, texts):
        rate, _ = self.get_parameter("sample_rate", 1)
        if stream.frame_id % int(rate):
            return StreamEvent.DROP_FRAME, {}
        return StreamEvent.OKAY, {"texts": texts}


class TextTransform(PipelineElement):
    TRANSFORMS = {
        "lowercase": str.lower,
        "none": lambda t: t,
        "titlecase": str.title,
        "uppercase": str.upper,
    }

    def __init__(self, context):
        context.set_protocol("text_transform:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, texts):
        kind, found = self.get_parameter("transform")
        if not found:
            return StreamEvent.ERROR, {"diagnostic": 'Must provide "transform" parameter'}
        fn = self.TRANSFORMS.get(kind)
        if fn is None:
            return StreamEvent.ERROR, {"diagnostic": f"Unknown text transform type: {kind}"}
        return StreamEvent.OKAY, {"texts": texts if kind == "none" else [fn(t) for t in texts]}


class TextWriteFile(DataTarget):
    def __init__(self, context):
        context.set_protocol("text_write_file:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, texts):
        for text in texts:
            path = self.next_target_path(stream)
            try:
                Path(path).write_text(text)
            except Exception as exc:
                return StreamEvent.ERROR, {"diagnostic": f"Error saving text: {exc}"}
        return StreamEvent.OKAY, {}
