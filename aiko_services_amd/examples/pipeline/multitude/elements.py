"""Aliases of PE_Add used by the multi-process load-test pipelines
(reference ``examples/pipeline/multitude/elements.py``)."""
from aiko_services_amd.examples.pipeline.elements import PE_Add

__all__ = ["PE_A0", "PE_B0", "PE_C0"] + [f"PE_{i:03d}" for i in range(0, 100, 10)]

PE_A0 = type("PE_A0", (PE_Add,), {"__module__": __name__})
PE_B0 = type("PE_B0", (PE_Add,), {"__module__": __name__})
PE_C0 = type("PE_C0", (PE_Add,), {"__module__": __name__})
for _i in range(0, 100, 10):
    globals()[f"PE_{_i:03d}"] = type(f"PE_{_i:03d}", (PE_Add,), {"__module__": __name__})
