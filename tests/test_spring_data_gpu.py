"""Spring Data RedissonConnection.pfAdd/pfCount/pfMerge over the engine vs the oracle."""
import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import IllegalArgumentException
from redisson_amd.spring_data import RedissonConnection

pytestmark = pytest.mark.gpu


def test_pf_commands(client, fresh):
    conn = RedissonConnection(client)
    k1, k2, k3 = ((fresh + s).encode() for s in ("a", "b", "c"))
    rng = np.random.default_rng(1)
    e1 = [rng.bytes(12) for _ in range(3000)]
    e2 = e1[1000:] + [rng.bytes(7) for _ in range(2000)]
    assert conn.pfAdd(k1, *e1) == 1
    assert conn.pfAdd(k1, *e1[:50]) == 0
    assert conn.pfAdd(k2, *e2) == 1
    r1, r2 = O.hll_new(), O.hll_new()
    O.hll_pfadd(r1, *O.arena(e1))
    O.hll_pfadd(r2, *O.arena(e2))
    assert conn.pfCount(k1) == O.hll_count(r1)
    u = r1.copy()
    O.hll_merge(u, r2)
    assert conn.pfCount(k1, k2) == O.hll_count(u)
    conn.pfMerge(k3, k1, k2)
    assert conn.pfCount(k3) == O.hll_count(u)
    with pytest.raises(IllegalArgumentException):
        conn.pfCount()
    with pytest.raises(IllegalArgumentException):
        conn.pfCount(k1, None)


def test_pf_commands_binary_keys(client, fresh):
    """byte[] keys may hold any byte (RedissonConnection.java:2203): keys that differ only after a
    zero byte are distinct HLLs; the *_n entry points carry (bytes, length)."""
    conn = RedissonConnection(client)
    base = fresh.encode()
    ka, kb = base + b"\x00a", base + b"\x00b"
    rng = np.random.default_rng(2)
    ea = [rng.bytes(16) for _ in range(500)]
    eb = [rng.bytes(16) for _ in range(900)]
    assert conn.pfAdd(ka, *ea) == 1
    assert conn.pfAdd(kb, *eb) == 1
    ra, rb = O.hll_new(), O.hll_new()
    O.hll_pfadd(ra, *O.arena(ea))
    O.hll_pfadd(rb, *O.arena(eb))
    assert conn.pfCount(ka) == O.hll_count(ra)
    assert conn.pfCount(kb) == O.hll_count(rb)
    # the NUL-terminated form sees only the common prefix, which holds nothing
    assert client.getHyperLogLog(fresh).count() == 0
    conn.pfMerge(base + b"\x00\xff", ka, kb)
    u = ra.copy()
    O.hll_merge(u, rb)
    assert conn.pfCount(base + b"\x00\xff") == O.hll_count(u)
