"""rccl_check.py -- librbx's RCCL merge inside a PyTorch process, the way bench.py's C4 leg runs it
at N > 1 (torch.distributed over RCCL initialised first, then librbx's own communicator from a
unique id broadcast through torch.distributed), here with one rank: every call of the N-rank path
(unique id, init, info, pack -> ncclAllReduce(u8, max) -> unpack) executes on the GPU.

    python tools/rccl_check.py      -> one JSON line; exit 0 iff the registers survive the merge
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from redisson_amd import RedissonClient, device_keys  # noqa: E402
from redisson_amd import _lib as L  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    client = RedissonClient(0)
    nh, per = 64, 4096
    hs = []
    for i in range(nh):
        hp = C.c_void_p()
        assert L.lib().rbx_hll_open(client.ctx, f"rc-{i}".encode(), 1, C.byref(hp)) == 0
        hs.append(hp.value)
    arr = (C.c_void_p * nh)(*hs)
    el = torch.randint(0, 256, (nh * per, 16), dtype=torch.uint8, device="cuda")
    seg = np.arange(nh + 1, dtype=np.uint64) * np.uint64(per)
    changed = torch.zeros(nh, dtype=torch.int32, device="cuda")
    dk = device_keys(el.data_ptr(), nh * per, 16)
    assert L.lib().rbx_hll_add_multi_dev(client.ctx, arr, nh, None, seg.ctypes.data_as(L.u64p), C.byref(dk),
                                         changed.data_ptr(), None) == 0, L.last_error()
    L.lib().rbx_synchronize(client.ctx)
    before = np.zeros(nh, np.uint64)
    assert L.lib().rbx_hll_count_each_handles(client.ctx, arr, nh, before.ctypes.data_as(L.u64p)) == 0

    uid = (C.c_uint8 * 128)()
    assert L.lib().rbx_rccl_unique_id(uid) == 0
    obj = [bytes(uid)]
    dist.broadcast_object_list(obj, src=0)
    uid = (C.c_uint8 * 128).from_buffer_copy(obj[0])
    assert L.lib().rbx_rccl_init(client.ctx, uid, 1, 0) == 0, L.last_error()
    nr, rk = C.c_int(), C.c_int()
    assert L.lib().rbx_rccl_info(client.ctx, C.byref(nr), C.byref(rk)) == 0
    assert L.lib().rbx_hll_allreduce_max(client.ctx, arr, nh) == 0, L.last_error()
    L.lib().rbx_synchronize(client.ctx)
    after = np.zeros(nh, np.uint64)
    assert L.lib().rbx_hll_count_each_handles(client.ctx, arr, nh, after.ctypes.data_as(L.u64p)) == 0
    ok = bool(np.array_equal(before, after)) and nr.value == 1 and rk.value == 0
    print(json.dumps({"check": "rccl_in_torch_process", "nranks": nr.value, "rank": rk.value,
                      "hlls": nh, "counts_unchanged": ok, "mean_count": float(after.mean())}), flush=True)
    dist.destroy_process_group()
    client.shutdown()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
