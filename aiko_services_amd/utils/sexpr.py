"""S-expression codec — the wire format of every control-plane message.

Wire-compatible with the reference codec (``main/utilities/parser.py:85-227``):

* ``generate("cmd", [a, b])`` -> ``"(cmd a b)"``; dicts become ``key: value`` pairs; strings
  containing whitespace / parentheses, or that start with ``N:``, are emitted in canonical
  form ``len:data``; ``None`` is ``0:``; the empty string is ``""``; nested lists/tuples/dicts
  recurse; every other value is rendered with ``str()``.
* ``parse(payload)`` -> ``(car, cdr)``; canonical ``len:data`` and quoted ``'..'``/``".."``
  tokens are accepted at token start; a list whose first element is a ``key:`` symbol becomes
  a dict; all scalars decode as ``str`` (callers coerce, e.g. :func:`parse_int`).

The implementation is a single-pass index scanner (no per-character regex, no recursion
on sub-strings), which matters because every actor message and every ``process_frame``
metadata record passes through it.  The native module ``aiko_services_amd/_sexpr.so``
(``csrc/host/sexpr.c``, built by ``csrc/build.py``) implements the same scanner, dict
conversion and generator in C and is used when present (``AIKO_SEXPR_NATIVE=0`` forces the
Python code below, which stays the reference: ``tests/test_sexpr_native.py`` fuzzes one
against the other).
"""
from __future__ import annotations

import os
from typing import Any

try:
    from .. import _sexpr as _native          # csrc/host/sexpr.c
except ImportError:                           # not built (source checkout before build())
    _native = None
if os.environ.get("AIKO_SEXPR_NATIVE", "1") == "0":
    _native = None

__all__ = ["generate", "parse", "parse_float", "parse_int", "parse_number",
           "generate_s_expression", "parse_list_to_dict"]

_WS = " \t\n\r"
_TENSOR_MAGIC = b"\x00AIKO-TP1\n"          # message/tensor_payload.py MAGIC
_DELIMS = set(" \t\n\r()")


def _needs_canonical(s: str) -> bool:
    if not s:
        return False
    for ch in s:
        if ch in _DELIMS:
            return True
    # leading "digits:" would be mistaken for a canonical length prefix
    i = 0
    n = len(s)
    while i < n and s[i].isdigit():
        i += 1
    return 0 < i < n and s[i] == ":"


def _dict_to_list(d: dict) -> list:
    out = []
    for k, v in d.items():
        out.append(f"{k}:")
        out.append(v)
    return out


def _gen(expr, parts: list) -> None:
    parts.append("(")
    first = True
    for el in expr:
        if not first:
            parts.append(" ")
        first = False
        if el is None:
            parts.append("0:")
        elif isinstance(el, str):
            if el == "":
                parts.append('""')
            elif _needs_canonical(el):
                parts.append(f"{len(el)}:{el}")
            else:
                parts.append(el)
        elif isinstance(el, dict):
            _gen(_dict_to_list(el), parts)
        elif isinstance(el, (list, tuple)):
            _gen(el, parts)
        elif isinstance(el, (int, float)):
            parts.append(str(el))
        else:
            _refuse_array(el)
            parts.append(str(el))
    parts.append(")")


def _refuse_array(el) -> None:
    """Arrays never become text: ``str(tensor)`` is lossy and unparseable (send them with
    ``message.tensor_payload.encode_message``)."""
    if hasattr(el, "__dlpack__") or hasattr(el, "__array_interface__") \
            or getattr(type(el), "__aiko_device_result__", False):
        raise TypeError(f"generate(): cannot render {type(el).__name__} as an S-expression "
                        "(use message.tensor_payload.encode_message)")


def generate_s_expression(expression) -> str:
    if _native is not None:
        return _native.generate(expression)
    return _generate_py(expression)


def _generate_py(expression) -> str:
    parts: list = []
    _gen(expression, parts)
    return "".join(parts)


def generate(command: str, parameters) -> str:
    """``generate("add", ["a", 1])`` -> ``"(add a 1)"``."""
    if isinstance(parameters, dict):
        parameters = _dict_to_list(parameters)
    elif isinstance(parameters, tuple):
        parameters = list(parameters)
    elif parameters is None:
        parameters = []
    return generate_s_expression([command] + list(parameters))


class _Scanner:
    __slots__ = ("s", "n", "i")

    def __init__(self, s: str):
        self.s = s
        self.n = len(s)
        self.i = 0

    def canonical(self):
        """At token start: ``digits:data`` -> (True, token) else (False, None)."""
        s, i, n = self.s, self.i, self.n
        j = i
        while j < n and "0" <= s[j] <= "9":
            j += 1
        if j == i or j >= n or s[j] != ":" or j + 1 >= n:
            return False, None
        length = int(s[i:j])
        start = j + 1
        if length == 0:
            self.i = start
            return True, None
        self.i = start + length
        return True, s[start:start + length]

    def quoted(self):
        s, i = self.s, self.i
        q = s[i]
        if q != '"' and q != "'":
            return False, None
        end = s.find(q, i + 1)
        if end < 0:
            return False, None
        self.i = end + 1
        return True, s[i + 1:end]

    def parse_list(self) -> list:
        """Parse until the matching ')' (or end); the opening '(' already consumed."""
        s, n = self.s, self.n
        result: list = []
        token_start = -1
        while self.i < n:
            if token_start < 0:
                ok, tok = self.canonical()
                if ok:
                    result.append(tok)
                    continue
                ok, tok = self.quoted()
                if ok:
                    result.append(tok)
                    continue
            c = s[self.i]
            if c == "(":
                if token_start >= 0:
                    result.append(s[token_start:self.i])
                    token_start = -1
                self.i += 1
                result.append(self.parse_list())
                continue
            if c == ")":
                if token_start >= 0:
                    result.append(s[token_start:self.i])
                self.i += 1
                return result
            if c in _WS:
                if token_start >= 0:
                    result.append(s[token_start:self.i])
                    token_start = -1
            elif token_start < 0:
                token_start = self.i
            self.i += 1
        if token_start >= 0:
            result.append(s[token_start:])
        return result


def parse(payload, dictionaries_flag: bool = True):
    """``"(cmd a (b c) k: v)"`` -> ``("cmd", ["a", ["b", "c"], ...])``."""
    if isinstance(payload, (bytes, bytearray, memoryview)):
        if bytes(payload[:len(_TENSOR_MAGIC)]) == _TENSOR_MAGIC:
            from ..message.tensor_payload import decode_message
            return decode_message(payload)          # binary message with arrays (tensor_payload)
        payload = bytes(payload).decode("utf-8")
    result = _native.scan(payload) if _native is not None else _Scanner(payload).parse_list()
    car, cdr = "", []
    if result:
        head = result[0]
        if isinstance(head, str):
            car = head
        elif isinstance(head, list) and head:
            car = head[0]
            cdr = head[1:]
    if dictionaries_flag:
        cdr = parse_list_to_dict(cdr)
    return car, cdr


def parse_list_to_dict(tree: Any):
    if _native is not None:
        return _native.to_dict(tree)
    return _to_dict_py(tree)


def _to_dict_py(tree: Any):
    if isinstance(tree, list) and tree:
        car = tree[0]
        if isinstance(car, str) and car.endswith(":"):
            if len(tree) % 2:
                raise ValueError(f'Error parsing S-Expression dictionary starting at keyword "{car}", '
                                 "must have pairs of keywords and values")
            out = {}
            for i in range(0, len(tree), 2):
                key = tree[i]
                if not isinstance(key, str):
                    raise ValueError(f'Error parsing S-Expression dictionary starting at keyword "{key}", '
                                     "keyword must be a string")
                if key and not key.endswith(":"):
                    raise ValueError(f'Error parsing S-Expression dictionary starting at keyword "{key}", '
                                     'keyword must end with ":" character')
                out[key[:-1]] = _to_dict_py(tree[i + 1])
            return out
        return [_to_dict_py(e) for e in tree]
    return tree


def parse_int(payload, default: int = 0) -> int:
    try:
        return int(payload)
    except (TypeError, ValueError):
        return default


def parse_float(payload, default: float = 0.0) -> float:
    try:
        return float(payload)
    except (TypeError, ValueError):
        return default


def parse_number(payload, default=0):
    try:
        return int(payload)
    except (TypeError, ValueError):
        try:
            return float(payload)
        except (TypeError, ValueError):
            return default
