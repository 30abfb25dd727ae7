#!/usr/bin/env python3
"""Diagnostic only (never a reported number): how much of the ResNet-50 bench's wall time a
kernel costs once the two frame lanes overlap, by replacing it with a no-op in this process
and re-running the bench.  python scripts/sensitivity.py <fc|stem|gap|none> [bench args]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    what = sys.argv[1]
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import vision as V
    if what == "fc":
        C.linear = lambda x, spec, out=None, residual=None: out
    elif what == "stem":
        C.stem_pool_u8 = lambda frames, spec, mean, std, out=None, variant=None: out
    elif what == "gap":
        V.avgpool = lambda x, out=None: out
    import bench
    bench.main(sys.argv[2:])


if __name__ == "__main__":
    main()
