#!/usr/bin/env python3
"""FETCH_SIZE calibration on a known byte count (MI355X_MICROARCH.md: other
access widths are uncalibrated): torch's vectorised copy of a 512 MiB fp32
tensor (16 B per lane loads), run under rocprofv3 --pmc FETCH_SIZE next to the
kernel being priced.  Reads per copy: exactly 512 MiB."""
import torch

a = torch.randn(8192 * 8192 * 2, device="cuda")
b = torch.empty_like(a)
for _ in range(8):
    b.copy_(a)
torch.cuda.synchronize()
print("copied", a.numel() * 4, "bytes x 8")
