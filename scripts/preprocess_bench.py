#!/usr/bin/env python3
"""Time the ResNet pre-processing kernel alone (uint8 224x224 frames -> zero-bordered bf16 stem input)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from aiko_services_amd.models.resnet50 import ResNet50
    from aiko_services_amd.ops import require_native
    require_native()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    m = ResNet50(device="cuda")
    x = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda")
    fn = (lambda: m.preprocess(x)) if hasattr(m, "preprocess") else None
    if fn is None:
        raise SystemExit("ResNet50 has no preprocess()")
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"preprocess B={B}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us")


if __name__ == "__main__":
    main()
