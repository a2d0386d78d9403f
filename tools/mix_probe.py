"""mix_probe.py -- do random reads and streaming writes share one request budget?

Runs the random-gather probe (k_gather_probe, 512 MiB table) and the stream-write probe
(k_stream_write) alone and then concurrently on two streams, and prints one JSON line: if the
concurrent time is near the sum of the two, reads and writes draw on one shared limit (the
request-time floor of bench.py's request_frac adds them); near the max, they overlap.

    python tools/mix_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from redisson_amd import RedissonClient  # noqa: E402
from redisson_amd import _lib as L  # noqa: E402


def main():
    client = RedissonClient(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    table = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    table.random_(0, 255, generator=g)
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    wbuf = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
    nkeys, k = 50_000_000, 7

    def gather(st):
        L.lib().rbx_bench_gather(client.ctx, table.data_ptr(), table.numel(), nkeys, k, sink.data_ptr(), st.cuda_stream)

    def write(st):
        L.lib().rbx_bench_stream_write(client.ctx, wbuf.data_ptr(), wbuf.numel(), st.cuda_stream)

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(torch.cuda.current_stream())
            fn()
            # join both streams back into the timing stream
            for st in (s1, s2):
                ev = torch.cuda.Event()
                ev.record(st)
                torch.cuda.current_stream().wait_event(ev)
            e1.record(torch.cuda.current_stream())
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best

    def start_both():
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        s1.wait_event(ev)
        s2.wait_event(ev)

    t_g = timed(lambda: (start_both(), gather(s1)))
    t_w = timed(lambda: (start_both(), write(s2)))
    t_both = timed(lambda: (start_both(), gather(s1), write(s2)))
    reads = nkeys * k
    writes = wbuf.numel() / 64
    print(json.dumps({"probe": "mix", "gather_ms": t_g, "write_ms": t_w, "both_ms": t_both,
                      "sum_ms": t_g + t_w, "max_ms": max(t_g, t_w),
                      "read_requests_per_s_alone": reads / (t_g / 1e3),
                      "write_requests_per_s_alone": writes / (t_w / 1e3),
                      "requests_per_s_both": (reads + writes) / (t_both / 1e3)}), flush=True)
    client.shutdown()


if __name__ == "__main__":
    main()
