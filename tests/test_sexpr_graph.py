"""S-expression codec and graph utilities (reference self-tests ``utilities/parser.py:229-248``,
``utilities/graph.py:1-24``)."""
import pytest

from aiko_services_amd.utils.graph import Graph, Node
from aiko_services_amd.utils.sexpr import generate, parse, parse_float, parse_int, parse_number

GOLDEN = [
    ("(a 0: b)", "a", [None, "b"]),
    ("(a b ())", "a", ["b", []]),
    ("(a b (c d))", "a", ["b", ["c", "d"]]),
    ("(a b (c d) (e f (g h)))", "a", ["b", ["c", "d"], ["e", "f", ["g", "h"]]]),
    ("(a b: 1 c: 2)", "a", {"b": "1", "c": "2"}),
    ("(a b: 1 c: (d e))", "a", {"b": "1", "c": ["d", "e"]}),
    ("(a b: 1 c: (d: 1 e: 2))", "a", {"b": "1", "c": {"d": "1", "e": "2"}}),
    ("(7:a b c d)", "a b c d", []),
    ("(3:a b 3:c d)", "a b", ["c d"]),
]


@pytest.mark.parametrize("payload,car,cdr", GOLDEN)
def test_parse_golden(payload, car, cdr):
    c, d = parse(payload)
    assert c == car
    assert d == cdr


@pytest.mark.parametrize("payload,car,cdr", GOLDEN)
def test_round_trip(payload, car, cdr):
    out = generate(car, cdr)
    assert parse(out) == (car, cdr)


def test_generate_forms():
    assert generate("add", ["a", 1, 2.5, True]) == "(add a 1 2.5 True)"
    assert generate("x", {"k": "v", "n": 3}) == "(x k: v n: 3)"
    assert generate("x", ["has space", "(paren", "12:ab"]) == "(x 9:has space 6:(paren 5:12:ab)"
    assert generate("x", [None, ""]) == '(x 0: "")'
    assert generate("process_frame", ({"stream_id": 1, "frame_id": 0}, {"a": 0})) == \
        "(process_frame (stream_id: 1 frame_id: 0) (a: 0))"
    assert generate("c", [["a", ["b"]], ()]) == "(c (a (b)) ())"


def test_parse_quoted_and_misc():
    assert parse("(a 'b c' \"d e\")") == ("a", ["b c", "d e"])
    assert parse("abc") == ("abc", [])
    assert parse("(process_frame (stream_id: 1 frame_id: 7) (a: 0))") == \
        ("process_frame", [{"stream_id": "1", "frame_id": "7"}, {"a": "0"}])
    assert parse(b"(x y)") == ("x", ["y"])
    with pytest.raises(ValueError):
        parse("(a b: 1 c:)")


def test_parse_numbers():
    assert parse_int("12") == 12 and parse_int("x", 3) == 3
    assert parse_float("1.5") == 1.5 and parse_float("?", 2.0) == 2.0
    assert parse_number("3") == 3 and parse_number("3.5") == 3.5 and parse_number("z", -1) == -1


def test_graph_traverse_diamond_and_properties():
    props = []
    heads, succ = Graph.traverse(["(A (B D (x: y)) (C D))"], lambda n, p, pr: props.append((n, p, pr)))
    assert list(heads) == ["A"]
    assert list(succ["A"]) == ["B", "C"]
    assert list(succ["B"]) == ["D"] and list(succ["C"]) == ["D"]
    assert props == [("D", {"x": "y"}, "B")]
    g = Graph(heads)
    for name in succ:
        g.add(Node(name, None, succ[name]))
    assert [n.name for n in g.get_path()] == ["A", "B", "C", "D"]
    assert [n.name for n in g.iterate_after("B")] == ["C", "D"]


def test_graph_paths_and_multiple_heads():
    heads, succ = Graph.traverse(["(PE_IN_0 PE_TEXT PE_OUT)", "(PE_IN_1 PE_OUT)"])
    g = Graph(heads)
    for name in succ:
        g.add(Node(name, None, succ[name]))
    assert [n.name for n in g.get_path("PE_IN_1")] == ["PE_IN_1", "PE_OUT"]
    assert [n.name for n in g.get_path()] == ["PE_IN_0", "PE_TEXT", "PE_OUT"]
    assert Graph.path_local("a:b") == "a" and Graph.path_remote("a:b") == "b"
    assert Graph.path_local(":b") is None and Graph.path_remote("a") is None
    with pytest.raises(KeyError):
        g.add(Node("PE_OUT"))


def test_graph_reference_order_chain_with_revisit():
    # "(PE_0 PE_1 (PE_2 PE_1))": PE_1 re-visited via PE_2 must move after PE_2
    heads, succ = Graph.traverse(["(PE_0 PE_1 (PE_2 PE_1))"])
    g = Graph(heads)
    for name in succ:
        g.add(Node(name, None, succ[name]))
    assert [n.name for n in g.get_path()] == ["PE_0", "PE_2", "PE_1"]


def test_dashboard_plugin_pages():
    """tools/dashboard plugins: lookup by service name / protocol; registrar + GPU pages."""
    from aiko_services_amd.tools import dashboard as D
    svc = ["aiko/host/10/1", "registrar", "au/registrar:2", "mqtt", "root", []]
    gpu = ["aiko/host/11/2", "yolo", "au/pipeline:0", "mqtt", "root", ["ec=true"]]

    class Fake:
        variables = {"gpu_fps": "20000", "hbm_pool_mb": "512", "lifecycle": "ready"}
        flat_variables = D.Dashboard.flat_variables

        def services(self):
            return [svc, gpu]
    assert D.find_plugin(svc) is D.registrar_page
    assert D.find_plugin(gpu) is None
    lines = D.registrar_page(Fake(), svc)
    assert len(lines) == 3 and "aiko/host/11/2" in lines[2]
    g = D.gpu_page(Fake(), gpu)
    assert any("gpu_fps" in r for r in g) and not any("lifecycle" in r for r in g)
    D.register_plugin("yolo", D.gpu_page)
    assert D.find_plugin(gpu) is D.gpu_page
    del D.PLUGINS["yolo"]


def test_dashboard_log_level_popup():
    """LogLevelPopupMenu: starts on the service's level, arrows/digits pick, enter publishes
    (update log_level LEVEL) through the dashboard's edit path; escape cancels."""
    from aiko_services_amd.tools import dashboard as D
    sent = []

    class Fake:
        variables = {"log_level": "WARNING"}

        def edit_variable(self, name, value):
            sent.append((name, value))
    menu = D.LogLevelPopupMenu(Fake())
    assert menu.levels[menu.index] == "WARNING"
    assert menu.key(258) is None and menu.key(10) == menu.levels[(menu.levels.index("WARNING") + 1) % len(menu.levels)]
    assert sent[-1][0] == "log_level"
    assert D.LogLevelPopupMenu(Fake()).key(ord("1")) == D.LOG_LEVELS[0]
    assert D.LogLevelPopupMenu(Fake()).key(27) == "" and len(sent) == 2


def test_gstreamer_launch_descriptions_and_gating():
    """elements/gstreamer: reference launch strings; without the Gst typelib the readers and
    writers raise GStreamerError (no silent fallback)."""
    import pytest
    from aiko_services_amd.elements import gstreamer as G
    assert G.file_reader_launch("a.mp4").startswith("filesrc location=a.mp4 ! qtdemux ! avdec_h264")
    assert "appsink name=sink" in G.camera_reader_launch("/dev/video0")
    assert "udpsink host=h port=5000" in G.stream_writer_launch("h", 5000)
    assert "rtmpsink" in G.stream_writer_launch("h", 5000, "rtmp://x/y")
    assert "framerate=25/1" in G.file_writer_launch("o_%02d.mp4", 640, 480, 25)
    assert "rtph264depay" in G.stream_reader_launch("0.0.0.0", 6000)
    try:
        G.gst_initialise()
        available = True
    except G.GStreamerError:
        available = False
    if not available:
        with pytest.raises(G.GStreamerError):
            G.VideoFileReader("missing.mp4")
