#!/usr/bin/env python3
"""Plain device-to-device copies of a few sizes (torch copy_), for rocprofv3 kernel traces:
the small-batch floor a streaming kernel of the same bytes is compared with."""
import torch

dev = torch.device("cuda", 0)
for mb in (8, 32, 128):
    n = mb << 19   # uint16 elements
    a = torch.randint(0, 4096, (n,), dtype=torch.int16, device=dev)
    b = torch.empty_like(a)
    for _ in range(30):
        b.copy_(a)
torch.cuda.synchronize()
print("ok")
