"""``aiko`` command-line front-end (the reference's legacy ``aiko`` CLI, ``main/cli.py``, was
disabled; BASELINE's north star names ``aiko pipeline create``).

    aiko pipeline create|destroy ...   (= aiko_pipeline)
    aiko registrar                     (= aiko_registrar)
    aiko dashboard [--snapshot]        (= aiko_dashboard)
    aiko broker [--port 1883]          in-repo MQTT broker (replaces mosquitto)
    aiko recorder [filter]
    aiko storage start|test_command|test_request
    aiko lifecycle manager N | client ID TOPIC
    aiko ec-test sc_test | ec_test [PID [SID [FILTER]]]   EC share / ServicesCache self tests
                                       (also: aiko share ..., the reference's command name)
    aiko echo-bench                    BASELINE config 1 (two-process echo pipeline)
    aiko bench ...                     bench.py (ResNet-50 pipeline on MI355X)
    aiko build                         compile the HIP/C++ library for gfx950
"""
from __future__ import annotations

import sys


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    if cmd == "pipeline":
        from ..pipeline.cli import main as m
        return m(args=rest, standalone_mode=True)
    if cmd == "registrar":
        from ..control.registrar import main as m
    elif cmd == "dashboard":
        from .dashboard import main as m
    elif cmd == "broker":
        from ..message.mqtt_broker import main as m
    elif cmd == "recorder":
        from .recorder import main as m
    elif cmd == "storage":
        from .storage import main as m
    elif cmd == "lifecycle":
        from ..control.lifecycle import main as m
    elif cmd in ("ec-test", "share"):
        from .ec_test import main as m
    elif cmd == "echo-bench":
        from .echo_bench import main as m
    elif cmd == "bench":
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
        from bench import main as m
    elif cmd == "build":
        from ..csrc.build import main as m
    else:
        print(f"aiko: unknown command {cmd!r}\n{__doc__}")
        return 2
    return m(rest)


if __name__ == "__main__":
    sys.exit(main())
