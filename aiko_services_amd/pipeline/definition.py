"""PipelineDefinition parsing and validation (reference ``main/pipeline.py:138-178,896-973``
and the in-source Avro schema ``:1323-1440``).

No avro on the boxes, so the schema is enforced by a small hand-written validator with the
same rules: required ``version`` (int, must be 0), ``name``, ``runtime`` (enum go|python,
must be python), ``graph`` (array of S-expression strings), optional ``parameters`` (map of
bool|int|null|string), ``elements`` (each: ``name``, ``input``/``output`` arrays of
{name, type}, optional ``parameters``, ``deploy`` with exactly one of ``local``
{module, class_name?} or ``remote`` {module, service_filter{topic_path,name,owner,protocol,
transport,tags}}); ``"#"`` keys are comments and discarded.

MI355X extension (optional, every reference JSON stays valid): ``deploy.local.device``
(e.g. ``"gpu:3"`` / ``"cuda:0"``), ``deploy.local.dtype``, ``deploy.local.stage`` (pipeline-
parallel stage index) and a pipeline-level ``"parallel": {"mode": "pp"|"dp", "gpus": N}``.
"""
from __future__ import annotations

import copy
import json
from dataclasses import dataclass, field
from typing import Dict, List

__all__ = ["PipelineDefinition", "PipelineElementDefinition", "PipelineElementDeployLocal",
           "PipelineElementDeployRemote", "DefinitionError", "parse_pipeline_definition",
           "parse_pipeline_definition_dict", "validate_definition", "PIPELINE_DEFINITION_VERSION"]

PIPELINE_DEFINITION_VERSION = 0
COMMENT = "#"


class DefinitionError(ValueError):
    pass


@dataclass
class PipelineElementDeployLocal:
    module: str
    class_name: str = None
    device: str = None
    dtype: str = None
    stage: int = None


@dataclass
class PipelineElementDeployRemote:
    module: str
    service_filter: Dict[str, str]


@dataclass
class PipelineElementDefinition:
    name: str
    input: List[Dict[str, str]]
    output: List[Dict[str, str]]
    parameters: Dict = field(default_factory=dict)
    deploy: object = None


@dataclass
class PipelineDefinition:
    version: int
    name: str
    runtime: str
    graph: List[str]
    parameters: Dict
    elements: List
    parallel: Dict = None
    map_in_nodes: Dict = field(default_factory=dict)
    map_out_nodes: Dict = field(default_factory=dict)


def _req(d, key, types, where):
    if key not in d:
        raise DefinitionError(f"{where}: missing required field '{key}'")
    if not isinstance(d[key], types) or (types is int and isinstance(d[key], bool)):
        raise DefinitionError(f"{where}: field '{key}' has wrong type {type(d[key]).__name__}")
    return d[key]


def _io_list(v, where):
    if not isinstance(v, list):
        raise DefinitionError(f"{where}: must be an array")
    for i, item in enumerate(v):
        if not isinstance(item, dict):
            raise DefinitionError(f"{where}[{i}]: must be a record")
        for k in ("name", "type"):
            if not isinstance(item.get(k), str):
                raise DefinitionError(f"{where}[{i}]: '{k}' must be a string")


def _parameters(v, where):
    if not isinstance(v, dict):
        raise DefinitionError(f"{where}: parameters must be a map")
    for k, val in v.items():
        if k == COMMENT:
            continue
        if not (val is None or isinstance(val, (bool, int, str, float))):
            raise DefinitionError(f"{where}: parameter '{k}' must be boolean|int|null|string")


def validate_definition(d: dict) -> None:
    if not isinstance(d, dict):
        raise DefinitionError("PipelineDefinition must be a JSON object")
    _req(d, "version", int, "PipelineDefinition")
    _req(d, "name", str, "PipelineDefinition")
    runtime = _req(d, "runtime", str, "PipelineDefinition")
    if runtime not in ("go", "python"):
        raise DefinitionError(f"PipelineDefinition: runtime must be one of go|python, not {runtime}")
    graph = _req(d, "graph", list, "PipelineDefinition")
    if not all(isinstance(g, str) for g in graph):
        raise DefinitionError("PipelineDefinition: graph must be an array of strings")
    if "parameters" in d:
        _parameters(d["parameters"], "PipelineDefinition")
    elements = _req(d, "elements", list, "PipelineDefinition")
    for i, e in enumerate(elements):
        where = f"PipelineDefinition.elements[{i}]"
        if not isinstance(e, dict):
            raise DefinitionError(f"{where}: must be a record")
        name = _req(e, "name", str, where)
        where = f"PipelineElement {name}"
        _io_list(_req(e, "input", list, where), f"{where}.input")
        _io_list(_req(e, "output", list, where), f"{where}.output")
        if "parameters" in e:
            _parameters(e["parameters"], where)
        deploy = _req(e, "deploy", dict, where)
        kinds = [k for k in deploy if k != COMMENT]
        if len(kinds) != 1 or kinds[0] not in ("local", "remote"):
            raise DefinitionError(f"{where}: deploy must be either local or remote")
        spec = deploy[kinds[0]]
        if not isinstance(spec, dict):
            raise DefinitionError(f"{where}: deploy.{kinds[0]} must be a record")
        _req(spec, "module", str, f"{where}.deploy.{kinds[0]}")
        if kinds[0] == "local":
            if "class_name" in spec and not isinstance(spec["class_name"], str):
                raise DefinitionError(f"{where}: class_name must be a string")
        else:
            sf = _req(spec, "service_filter", dict, f"{where}.deploy.remote")
            for k, v in sf.items():
                if k not in ("topic_path", "name", "owner", "protocol", "transport", "tags", COMMENT):
                    raise DefinitionError(f"{where}: unknown service_filter field '{k}'")
                if k != COMMENT and not isinstance(v, str):
                    raise DefinitionError(f"{where}: service_filter.{k} must be a string")
    if "parallel" in d:
        p = d["parallel"]
        if not isinstance(p, dict) or p.get("mode", "dp") not in ("dp", "pp", "none"):
            raise DefinitionError("PipelineDefinition: parallel must be {mode: dp|pp, gpus: N}")


def parse_pipeline_definition_dict(d: dict, source: str = "<dict>") -> PipelineDefinition:
    d = copy.deepcopy(d)
    validate_definition(d)
    d.pop(COMMENT, None)
    d.setdefault("parameters", {})
    d["parameters"].pop(COMMENT, None)
    if d["version"] != PIPELINE_DEFINITION_VERSION:
        raise DefinitionError(f"PipelineDefinition: Version must be 0, but is {d['version']}")
    if d["runtime"] != "python":
        raise DefinitionError(f'PipelineDefinition: Runtime must be "python", but is "{d["runtime"]}"')
    elements = []
    for e in d["elements"]:
        e.pop(COMMENT, None)
        params = e.get("parameters", {})
        params.pop(COMMENT, None)
        deploy = e["deploy"]
        deploy.pop(COMMENT, None)
        kind, spec = next(iter(deploy.items()))
        spec.pop(COMMENT, None)
        if kind == "local":
            dep = PipelineElementDeployLocal(module=spec["module"],
                                             class_name=spec.get("class_name", e["name"]),
                                             device=spec.get("device"), dtype=spec.get("dtype"),
                                             stage=spec.get("stage"))
        else:
            sf = {k: "*" for k in ("topic_path", "name", "owner", "protocol", "transport", "tags")}
            sf.update({k: v for k, v in spec["service_filter"].items() if k != COMMENT})
            dep = PipelineElementDeployRemote(module=spec["module"], service_filter=sf)
        elements.append(PipelineElementDefinition(name=e["name"], input=e["input"], output=e["output"],
                                                  parameters=params, deploy=dep))
    return PipelineDefinition(version=d["version"], name=d["name"], runtime=d["runtime"],
                              graph=d["graph"], parameters=d["parameters"], elements=elements,
                              parallel=d.get("parallel"))


def parse_pipeline_definition(pathname: str) -> PipelineDefinition:
    with open(pathname, "r") as f:
        d = json.load(f)
    try:
        return parse_pipeline_definition_dict(d, pathname)
    except DefinitionError as exc:
        raise DefinitionError(f"Error: Parsing PipelineDefinition: {pathname}\n{exc}") from None
