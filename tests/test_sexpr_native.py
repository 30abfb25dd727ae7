"""The native S-expression codec (``csrc/host/sexpr.c``) against the Python reference scanner /
generator of ``utils/sexpr.py``: identical trees, dicts, text and errors on fuzzed input."""
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from aiko_services_amd.utils import sexpr as S


@pytest.fixture(scope="module")
def native():
    from aiko_services_amd.csrc.build import build_host_modules
    build_host_modules(verbose=False)
    import importlib
    mod = importlib.import_module("aiko_services_amd._sexpr")
    return mod


_ALPHABET = st.sampled_from(list("ab01239:() \t\n'\"xT@/.-_") + ["é", "²", "漢"])
_TEXT = st.text(_ALPHABET, max_size=60)


def _outcome(fn, *args):
    try:
        return ("ok", fn(*args))
    except ValueError as exc:
        return ("ValueError", str(exc))


@settings(max_examples=600, deadline=None)
@given(_TEXT)
def test_scan_and_to_dict_match_python(native, text):
    py_tree = S._Scanner(text).parse_list()
    assert native.scan(text) == py_tree
    assert _outcome(native.to_dict, py_tree) == _outcome(S._to_dict_py, py_tree)


_SCALAR = st.one_of(st.none(), _TEXT, st.integers(-10**6, 10**6), st.floats(allow_nan=False), st.booleans())
_EXPR = st.recursive(_SCALAR, lambda inner: st.one_of(
    st.lists(inner, max_size=5), st.tuples(inner, inner),
    st.dictionaries(st.text(st.sampled_from(list("abk_1")), min_size=1, max_size=4), inner, max_size=4)),
    max_leaves=25)


@settings(max_examples=600, deadline=None)
@given(st.lists(_EXPR, max_size=6))
def test_generate_matches_python_and_round_trips(native, expr):
    text = native.generate(expr)
    assert text == S._generate_py(expr)
    assert native.scan(text) == S._Scanner(text).parse_list()


def test_hop_messages_round_trip(native):
    msg = S.generate("process_frames", (
        [{"stream_id": "s", "frame_id": 1, "hop_rank": 0}, {"stream_id": "s", "frame_id": 2, "hop_rank": 0}],
        [{"x": "T@0/1/0/float32/16", "t": "F@1.5"}, {"x": "T@0/1/1/float32/16x4", "s": "has space"}]))
    cmd, args = S.parse(msg)
    assert cmd == "process_frames"
    assert args[0][1] == {"stream_id": "s", "frame_id": "2", "hop_rank": "0"}
    assert args[1][1]["s"] == "has space" and args[1][0]["t"] == "F@1.5"


def test_errors_match(native):
    for bad in (["a:"], ["a:", "1", "b"], ["a:", "1", None, "2"], ["a:", "1", ["x"], "2"]):
        assert _outcome(native.to_dict, bad) == _outcome(S._to_dict_py, bad)
