#!/usr/bin/env python3
"""Debug: the Whisper encoder through a copy-in CapturedCall vs a static (per-address) one vs
eager, on the same inputs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from aiko_services_amd.gpu.element import CapturedCall
    from aiko_services_amd.models.whisper import WhisperEncoder
    from aiko_services_amd.ops import require_native
    require_native()
    m = WhisperEncoder("tiny", device="cuda")
    g = torch.Generator().manual_seed(0)
    xs = [(0.1 * torch.randn(2, 32000, generator=g)).cuda() for _ in range(3)]
    eager = [m.encode(x).clone() for x in xs]
    copyin = CapturedCall(m.encode, [xs[0]])
    got_c = [copyin(x).clone() for x in xs]
    static = [CapturedCall(m.encode, [x], static=True) for x in xs]
    got_s = [c.graph_replay().clone() for c in static]
    torch.cuda.synchronize()
    for i in range(3):
        print(i, "copy-in vs eager", (got_c[i].float() - eager[i].float()).abs().max().item(),
              "static vs eager", (got_s[i].float() - eager[i].float()).abs().max().item())


if __name__ == "__main__":
    main()
