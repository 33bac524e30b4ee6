#!/usr/bin/env python3
"""PCIe copy bandwidth of this box (host boundary of kv_validate: store upload, status and
record fetch): page-locked host <-> HBM, one copy vs the same bytes split over S streams.

    python tools/pcie_bw.py [GB]   (HSA_ENABLE_SDMA=0 selects blit-kernel copies)"""
import sys
import time

import torch

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
n = int(gb * (1 << 30))
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
h.fill_(1)
d.fill_(2)
torch.cuda.synchronize()
for direction in ("h2d", "d2h"):
    for S in (1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(S)]
        best = 1e9
        for rep in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            step = (n + S - 1) // S
            for i, s in enumerate(streams):
                a, e = i * step, min(n, (i + 1) * step)
                with torch.cuda.stream(s):
                    if direction == "h2d":
                        d[a:e].copy_(h[a:e], non_blocking=True)
                    else:
                        h[a:e].copy_(d[a:e], non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        print(f"{direction} {gb:.2f} GB streams={S}: {best * 1e3:.1f} ms, {n / best / 1e9:.1f} GB/s", flush=True)
