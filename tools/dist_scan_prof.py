"""Times the exchange's reorder + scan (rle_dist_offsets_device, csrc/rle_dist.hip) at the configs[3]
shapes, for rocprofv3 --kernel-trace: world 8 x 131072 sizes (1 M entries) and world 1 x 1 M.
Prints HIP-event averages too.   usage: python tools/dist_scan_prof.py"""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "c-filestorage-server-and-client_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rle_mi355x as R  # noqa: E402

out = {}
for world, n in ((8, 131072), (1, 1 << 20), (8, 4096)):
    g = torch.randint(0, 70000, (world * n,), dtype=torch.int64, device="cuda")
    o = torch.empty_like(g)
    ws = R.dist_workspace(n, g.device)
    R.dist_offsets(g, world, n, o, ws=ws)
    torch.cuda.synchronize()
    ref = g.view(world, n).t().reshape(-1)
    assert torch.equal(o, torch.cumsum(ref, 0) - ref)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        R.dist_offsets(g, world, n, o, ws=ws)
    b.record()
    torch.cuda.synchronize()
    out[f"{world}x{n}"] = round(a.elapsed_time(b) / 20 * 1e3, 2)
print(json.dumps({"scan_us_per_call (2 launches, events)": out}))
