"""Device-to-device copy ceiling on the box (torch copy_ of 249 MB, the C2 AND result size), beside the
serializer's 0.096 ms for the same bytes (read + write)."""
import time

import torch

n = 248942352
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty(n, dtype=torch.uint8, device="cuda")
a.fill_(1)
for _ in range(5):
    b.copy_(a)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    b.copy_(a)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 50
print(f"copy {n} B: {ms:.4f} ms, {2 * n / ms / 1e6:.0f} GB/s of read + write")
