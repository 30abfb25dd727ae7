"""Isolated timing of the log-mel op (one stream, nothing concurrent): B=16 clips of 30 s.
AIKO_LOGMEL_DFT=1 selects the former direct-DFT kernel for comparison."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from aiko_services_amd.ops import require_native
    require_native()
    from aiko_services_amd.ops import audio as AU
    B, N = 16, 16000 * 30
    audio = torch.randn(B, N, device="cuda") * 0.1
    filters = AU.mel_filters().cuda()
    F_ = N // AU.HOP
    rows = F_ + 2
    out = torch.empty(B * rows, 80, dtype=torch.bfloat16, device="cuda")
    work = torch.empty(B * F_ * 80, dtype=torch.float32, device="cuda")
    gmax = torch.empty(B, dtype=torch.int32, device="cuda")
    for _ in range(3):
        AU.log_mel(audio, filters, out, rows, 1, work=work, gmax=gmax, frames=F_)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        AU.log_mel(audio, filters, out, rows, 1, work=work, gmax=gmax, frames=F_)
    e1.record()
    torch.cuda.synchronize()
    mode = "direct DFT" if os.environ.get("AIKO_LOGMEL_DFT") == "1" else "FFT"
    print(f"log_mel B={B} x 30 s ({mode}): {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
