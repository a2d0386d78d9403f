"""C1 leg alone (for rocprofv3): tryInit(1e7, 0.01), add 1M 16-byte keys into a fresh filter and
contains 2M, `reps` times -- the calls bench.py's run_c1 times."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from redisson_amd import BloomHandle, RedissonClient, device_keys  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
client = RedissonClient(0)
g = torch.Generator(device="cuda")
g.manual_seed(0x5EED0001)
keys = torch.randint(0, 256, (1_000_000, 16), dtype=torch.uint8, device="cuda", generator=g)
probe = torch.cat([keys, torch.randint(0, 256, (1_000_000, 16), dtype=torch.uint8, device="cuda", generator=g)])
cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
for r in range(reps):
    f = client.getBloomFilter(f"c1-{r}")
    assert f.tryInit(10_000_000, 0.01)
    h = BloomHandle(client, f"c1-{r}")
    h.add_dev(device_keys(keys.data_ptr(), 1_000_000, 16), cnt.data_ptr(), stream=stream.cuda_stream)
    h.contains_dev(device_keys(probe.data_ptr(), 2_000_000, 16), cnt.data_ptr() + 8, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    h.close()
    f.delete()
client.shutdown()
print("c1 ok")
