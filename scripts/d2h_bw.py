"""Diagnostic: device->pinned-host copy bandwidth on one or several streams (HIP via torch)."""
import time
import torch

n = 256 << 20
src = torch.empty(n, dtype=torch.uint8, device="cuda").fill_(1)
for nstreams in (1, 2, 3, 4):
    dst = [torch.empty(n // nstreams, dtype=torch.uint8, pin_memory=True) for _ in range(nstreams)]
    ss = [torch.cuda.Stream() for _ in range(nstreams)]
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(nstreams):
            with torch.cuda.stream(ss[i]):
                dst[i].copy_(src[i * (n // nstreams):(i + 1) * (n // nstreams)], non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
    print(f"streams {nstreams}: {n / el / 1e9:.1f} GB/s", flush=True)
