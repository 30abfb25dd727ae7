"""Register / scratch budget of kernels whose counted `s_waitcnt vmcnt(N)` schedules break when the
compiler puts state in scratch (CPU: hipcc cross-compiles gfx950 device assembly, no GPU needed).

A scratch load is a VMEM op the kernel's own counts do not include.  Waiting for it drains every
DMA issued before it.  Round 6 found two such cases: bneck_fused's DMA marks, rounds 3-5,
`profiles/bneck_r6.md`; and a spill in the MX-fp8 residual GEMM.  These tests pin both at zero."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

KERNELS = Path(__file__).resolve().parents[1] / "aiko_services_amd" / "csrc" / "kernels"
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if Path("/opt/rocm/bin/hipcc").exists() else None)


def _device_asm(src: str, tmp_path: Path) -> str:
    out = tmp_path / (Path(src).stem + ".s")
    cmd = [HIPCC, "-std=c++17", "-O3", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-I", str(KERNELS),
           "--cuda-device-only", "-S", "-o", str(out), str(KERNELS / src)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return out.read_text()


def _functions(asm: str) -> dict:
    """mangled kernel name -> (ScratchSize, VGPRs, the function's text)"""
    res = {}
    for m in re.finditer(r"^(_Z[^:\s]+):(.*?)^; ScratchSize: (\d+)", asm, re.S | re.M):
        name, body, scratch = m.group(1), m.group(2), int(m.group(3))
        v = re.search(r"^; NumVgprs: (\d+)", body, re.M)
        res[name] = (scratch, int(v.group(1)) if v else -1, body)
    return res


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
@pytest.mark.parametrize("src,pattern,n_min", [
    ("bneck_fused.hip", "bneck_fused_kernel", 2),          # identity and projection blocks
    ("gemm_fp8.hip", "gemm_fp8_pers2_kernel", 10),         # every persistent fp8 GEMM variant
    ("conv_patchw.hip", "conv3x3_patchw_kernelILi28ELi32E", 1),   # the default patch pitch
])
def test_counted_wait_kernels_use_no_scratch(tmp_path, src, pattern, n_min):
    fns = {k: v for k, v in _functions(_device_asm(src, tmp_path)).items() if pattern in k}
    assert len(fns) >= n_min, sorted(fns)
    for name, (scratch, vgprs, body) in fns.items():
        assert scratch == 0, f"{name}: {scratch} B of scratch"
        assert "scratch_load" not in body and "scratch_store" not in body, name
        assert 0 < vgprs <= 256, (name, vgprs)
