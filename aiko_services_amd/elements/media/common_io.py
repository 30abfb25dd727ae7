"""DataSource / DataTarget base elements (reference ``elements/media/common_io.py:26-151``).

``data_sources``: S-expression list of ``file://`` URLs or paths; a ``{}`` in the file name is a
glob whose match becomes the file id.  One path -> a single ``create_frame``; otherwise a
frame-generator thread yields ``data_batch_size`` paths per frame at ``rate`` frames/s and
STOPs when exhausted.  ``data_targets``: a ``file://`` path, optionally formatted with a
running file id.  MI355X addition: the ``synthetic://`` scheme is handled by the GPU source
elements (:mod:`aiko_services_amd.elements.gpu`).
"""
from __future__ import annotations

import os
from pathlib import Path

from ...pipeline.engine import PipelineElement
from ...pipeline.stream import StreamEvent
from ...utils.sexpr import parse

__all__ = ["contains_all", "file_glob_difference", "DataSource", "DataTarget", "parse_data_urls"]


def contains_all(source: str, match: str) -> bool:
    return all(ch in source for ch in match)


def file_glob_difference(file_glob, filename):
    tokens = file_glob.split("*")
    start = tokens[0]
    end = tokens[1] if len(tokens) > 1 else ""
    if filename.startswith(start) and filename.endswith(end) and len(filename) >= len(start) + len(end):
        return filename[len(start):len(filename) - len(end)]
    return None


def parse_data_urls(data_sources: str):
    """``"(file://a b)"`` or ``"file://a"`` -> list of (scheme, path)."""
    if data_sources.strip().startswith("("):
        head, rest = parse(data_sources)
        urls = [head] + list(rest)
    else:
        urls = [data_sources]
    out = []
    for url in urls:
        scheme, sep, path = str(url).partition("://")
        out.append(("file", scheme) if not sep else (scheme, path))
    return out


class DataSource(PipelineElement):
    def start_stream(self, stream, stream_id, use_create_frame=True):
        data_sources, found = self.get_parameter("data_sources")
        if not found:
            return StreamEvent.ERROR, {"diagnostic": 'Must provide "data_sources" parameter'}
        paths = []
        for scheme, path in parse_data_urls(str(data_sources)):
            if scheme != "file":
                return StreamEvent.ERROR, {"diagnostic": 'DataSource scheme must be "file://"'}
            file_glob = "*"
            if contains_all(path, "{}"):
                file_glob = os.path.basename(path).replace("{}", "*")
                path = os.path.dirname(path)
            p = Path(path)
            if not p.exists():
                return StreamEvent.ERROR, {"diagnostic": f'path "{p}" does not exist'}
            if p.is_file():
                paths.append((p, None))
            elif p.is_dir():
                for q in sorted(p.glob(file_glob)):
                    fid = file_glob_difference(file_glob, q.name) if file_glob != "*" else None
                    paths.append((q, fid))
            else:
                return StreamEvent.ERROR, {"diagnostic": f'"{p}" must be a file or a directory'}
        if use_create_frame and len(paths) == 1:
            self.create_frame(stream, {"paths": [paths[0][0]]})
        else:
            stream.variables["source_paths_generator"] = iter(paths)
            rate, _ = self.get_parameter("rate", default=None)
            self.create_frames(stream, self.frame_generator, rate=float(rate) if rate else None)
        return StreamEvent.OKAY, {}

    def frame_generator(self, stream, frame_id):
        batch, _ = self.get_parameter("data_batch_size", default=1)
        batch = int(batch)
        paths = []
        for _ in range(batch):
            try:
                path, _fid = next(stream.variables["source_paths_generator"])
            except StopIteration:
                break
            path = Path(path)
            if not path.is_file():
                return StreamEvent.ERROR, {"diagnostic": f'path "{path}" must be a file'}
            paths.append(path)
        if paths:
            return StreamEvent.OKAY, {"paths": paths}
        return StreamEvent.STOP, {"diagnostic": "All frames generated"}


class DataTarget(PipelineElement):
    def start_stream(self, stream, stream_id):
        data_targets, found = self.get_parameter("data_targets")
        if not found:
            return StreamEvent.ERROR, {"diagnostic": 'Must provide file "data_targets" parameter'}
        scheme, sep, path = str(data_targets).partition("://")
        if not sep:
            path = scheme
        elif scheme != "file":
            return StreamEvent.ERROR, {"diagnostic": 'DataTarget scheme must be "file://"'}
        stream.variables["target_file_id"] = 0
        stream.variables["target_path"] = path
        return StreamEvent.OKAY, {}

    def next_target_path(self, stream):
        path = stream.variables["target_path"]
        if contains_all(path, "{}"):
            path = path.format(stream.variables["target_file_id"])
            stream.variables["target_file_id"] += 1
        return path
