#!/usr/bin/env python3
"""Repeats the C2 contains (partitioned pipeline, forced) and compares every call's count with
the direct kernel's: a nondeterministic count means lost or stray pairs.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from redisson_amd import BloomHandle, RedissonClient, device_keys  # noqa: E402
from redisson_amd import _lib as L  # noqa: E402

n = int(os.environ.get("RBX_DET_KEYS", "100000000"))
client = RedissonClient(0)
stream = torch.cuda.Stream()
sp = stream.cuda_stream
g = torch.Generator(device="cuda")
g.manual_seed(7)
keys = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
f = client.getBloomFilter("det")
f.tryInitRaw(1 << 32, 7)
h = BloomHandle(client, "det")
cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
h.add_dev(device_keys(keys.data_ptr(), n // 2, 32), cnt.data_ptr(), stream=sp)
dk = device_keys(keys.data_ptr(), n, 32)
L.lib().rbx_tune(b"contains_partition", 0)
h.contains_dev(dk, cnt.data_ptr() + 8, stream=sp)
L.lib().rbx_tune(b"contains_partition", 1)
for i in range(6):
    h.contains_dev(dk, cnt.data_ptr() + 16 + 8 * i, stream=sp)
torch.cuda.synchronize()
c = cnt.tolist()
print(json.dumps({"direct": c[1], "partitioned": c[2:8], "ok": all(x == c[1] for x in c[2:8])}))
L.lib().rbx_tune(b"contains_partition", 2)
