"""RHyperLogLog on the GPU vs the CPU oracle (register-exact, PFCOUNT-integer-exact).

Mirrors T/RedissonHyperLogLogTest.java and the Redis PFADD/PFCOUNT/PFMERGE semantics
[redis-7.2 hyperloglog.c, restated in oracle/rbx_oracle.c].
"""
import base64
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from redisson_amd import Arena, IllegalArgumentException, RedisException, hll_add_multi, hll_count_each

pytestmark = pytest.mark.gpu
G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
SEED = 0x5EED0000


def regs_of(h) -> np.ndarray:
    d = h.exportDense()
    assert d[:4] == b"HYLL" and d[4] == 0 and len(d) == 12304
    return O.hll_dense_unpack(d[16:])


# ---- T/RedissonHyperLogLogTest.java ---------------------------------------------------------
def test_add_all(client, fresh):
    log = client.getHyperLogLog(fresh)
    log.addAll([1, 2, 3])
    assert log.count() == 3


def test_add(client, fresh):
    log = client.getHyperLogLog(fresh)
    log.add(1)
    log.add(2)
    log.add(3)
    assert log.count() == 3


def test_merge(client, fresh):
    hll1 = client.getHyperLogLog(fresh + "1")
    assert hll1.add("foo") and hll1.add("bar") and hll1.add("zap") and hll1.add("a")
    hll2 = client.getHyperLogLog(fresh + "2")
    assert hll2.add("a") and hll2.add("b") and hll2.add("c") and hll2.add("foo")
    assert hll2.add("c") is False
    hll3 = client.getHyperLogLog(fresh + "3")
    hll3.mergeWith(fresh + "1", fresh + "2")
    assert hll3.count() == 6
    assert hll1.countWith(fresh + "2") == 6


def test_redis_doc_examples(client, fresh):
    h = client.getHyperLogLog(fresh)
    assert h.addAll(["1", "2", "3", "4", "5"]) is True
    assert h.count() == 5
    h.addAll(["6", "7", "8", "8", "9", "10"])
    assert h.count() == 10
    e = client.getHyperLogLog(fresh + "e")
    assert e.addAll([]) is True  # PFADD without elements creates the key -> 1
    assert e.addAll([]) is False
    assert e.count() == 0
    assert client.getHyperLogLog(fresh + "missing").count() == 0


# ---- register / count parity ------------------------------------------------------------------
@pytest.mark.parametrize("i", range(8))
def test_golden_registers_and_counts(client, fresh, i):
    e = G["hll"][i]
    n = e["n"]
    mat = np.random.default_rng(SEED + 4 * 1000003 + n).integers(0, 256, size=(n, 16), dtype=np.uint8)
    h = client.getHyperLogLog(fresh)
    h.addAll(Arena.fixed(mat) if n else [])
    dense = base64.b64decode(e["dense"])
    assert h.exportDense()[16:] == dense
    assert h.count() == e["count"]


@pytest.mark.parametrize("L", [8, 16, 32, 64, 0])
def test_parity_element_layouts(client, fresh, L):
    rng = np.random.default_rng(100 + L)
    if L:
        mat = rng.integers(0, 256, size=(200000, L), dtype=np.uint8)
        a = Arena.fixed(mat)
        ob, oo = O.fixed_arena(mat)
    else:
        elems = [rng.bytes(int(x)) for x in rng.integers(0, 120, size=50000)]
        a = Arena(elems)
        ob, oo = O.arena(elems)
    h = client.getHyperLogLog(fresh)
    assert h.addAll(a) is True
    regs = O.hll_new()
    O.hll_pfadd(regs, ob, oo)
    assert np.array_equal(regs_of(h), regs)
    assert h.count() == O.hll_count(regs)


def test_pfadd_pipeline_sequential_replies(client, fresh):
    """A batch of PFADD commands naming the same HLL several times: every reply must see
    the commands before it (in-order pipeline semantics)."""
    rng = np.random.default_rng(7)
    names = [fresh + s for s in ["a", "b", "a", "a", "c", "b", "a"]]
    pool = [rng.bytes(10) for _ in range(40)]
    elems, segs = [], [0]
    for i in range(len(names)):
        m = int(rng.integers(0, 12))
        elems += [pool[int(j)] for j in rng.integers(0, 40 if i < 4 else 20, size=m)]
        segs.append(len(elems))
    replies = hll_add_multi(client, names, np.array(segs, np.uint64), Arena(elems))
    refs, want = {}, []
    for s, nm in enumerate(names):
        created = nm not in refs
        r = refs.setdefault(nm, O.hll_new())
        sub = elems[segs[s]:segs[s + 1]]
        ch = O.hll_pfadd(r, *O.arena(sub)) if sub else 0
        want.append(int(bool(ch) or created))
    assert replies.tolist() == want
    for nm, r in refs.items():
        assert np.array_equal(regs_of(client.getHyperLogLog(nm)), r)


def test_count_each_and_union(client, fresh):
    rng = np.random.default_rng(8)
    names, refs = [], []
    for i in range(50):
        n = int(rng.integers(0, 20000))
        mat = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
        nm = f"{fresh}-{i}"
        client.getHyperLogLog(nm).addAll(Arena.fixed(mat) if n else [])
        r = O.hll_new()
        if n:
            O.hll_pfadd(r, *O.fixed_arena(mat))
        names.append(nm)
        refs.append(r)
    got = hll_count_each(client, names)
    assert got.tolist() == [O.hll_count(r) for r in refs]
    u = O.hll_new()
    for r in refs[:10]:
        O.hll_merge(u, r)
    assert client.getHyperLogLog(names[0]).countWith(*names[1:10]) == O.hll_count(u)
    client.getHyperLogLog(fresh + "dst").mergeWith(*names[:10])
    assert np.array_equal(regs_of(client.getHyperLogLog(fresh + "dst")), u)


def test_tau_branch_and_high_registers(client, fresh):
    """Registers equal to 51 (hllTau path, evaluated with glibc pow on the host) and
    imported dense registers up to 63."""
    rng = np.random.default_rng(9)
    for trial in range(20):
        regs = rng.integers(0, 20, size=16384, dtype=np.uint8)
        regs[rng.integers(0, 16384, size=int(rng.integers(1, 50)))] = 51
        if trial % 2:
            regs[rng.integers(0, 16384, size=5)] = 63
        s = b"HYLL" + bytes([0, 0, 0, 0]) + bytes([0, 0, 0, 0, 0, 0, 0, 0x80]) + O.hll_dense_pack(regs)
        h = client.getHyperLogLog(f"{fresh}-{trial}")
        h.importString(s)
        assert h.count() == O.hll_count(regs)


def test_cached_cardinality_semantics(client, fresh):
    # a valid cached card in the header is returned as is by PFCOUNT (like redis)
    regs = O.hll_new()
    O.hll_pfadd(regs, *O.arena([b"x", b"y"]))
    s = b"HYLL" + bytes(4) + (1234).to_bytes(8, "little") + O.hll_dense_pack(regs)
    h = client.getHyperLogLog(fresh)
    h.importString(s)
    assert h.count() == 1234
    assert h.exportDense()[8:16] == (1234).to_bytes(8, "little")
    h.add(b"z")  # changes a register -> cache invalidated -> recomputed
    O.hll_pfadd(regs, *O.arena([b"z"]))
    assert h.count() == O.hll_count(regs)


def _sparse_encode(regs: np.ndarray) -> bytes:
    """Redis sparse encoding (ZERO / XZERO / VAL opcodes) of registers <= 32."""
    out = bytearray()
    i = 0
    while i < 16384:
        v = int(regs[i])
        j = i
        while j < 16384 and regs[j] == v:
            j += 1
        run = j - i
        while run:
            if v == 0:
                if run > 64:
                    r = min(run, 16384)
                    out += bytes([0x40 | ((r - 1) >> 8), (r - 1) & 0xFF])
                else:
                    r = run
                    out.append((r - 1) & 0x3F)
            else:
                r = min(run, 4)
                out.append(0x80 | ((v - 1) << 2) | (r - 1))
            run -= r
        i = j
    return bytes(out)


def test_sparse_import(client, fresh):
    rng = np.random.default_rng(10)
    regs = O.hll_new()
    O.hll_pfadd(regs, *O.fixed_arena(rng.integers(0, 256, size=(300, 16), dtype=np.uint8)))
    s = b"HYLL" + bytes([1, 0, 0, 0]) + bytes([0] * 7 + [0x80]) + _sparse_encode(regs)
    h = client.getHyperLogLog(fresh)
    h.importString(s)
    assert np.array_equal(regs_of(h), regs)
    assert h.count() == O.hll_count(regs)


def _header(sparse: int, card: bytes) -> bytes:
    return b"HYLL" + bytes([sparse, 0, 0, 0]) + card


def test_export_sparse_as_stored(client, fresh):
    """PFADD creates sparse strings ([redis-7.2] createHLLObject); GET returns the sparse string
    as Redis built it, element by element (hllSparseSet, restated in oracle RedisHll)."""
    rng = np.random.default_rng(11)
    mat = rng.integers(0, 256, size=(300, 16), dtype=np.uint8)
    ref = O.RedisHll()
    ref.pfadd(*O.fixed_arena(mat))
    h = client.getHyperLogLog(fresh)
    h.addAll(Arena([bytes(r) for r in mat]))
    s = h.exportString()
    assert s == ref.string(h.exportDense()[8:16])
    assert s[4] == 1 and h.exportString("sparse") == s
    assert np.array_equal(O.hll_sparse_unpack(s[16:]), ref.regs)
    # SET of the exported string round-trips (and keeps the sparse encoding)
    g = client.getHyperLogLog(fresh + "c")
    g.importString(s)
    assert g.exportString() == s and np.array_equal(regs_of(g), ref.regs)
    assert g.count() == h.count() == O.hll_count(ref.regs)
    g.delete()
    h.delete()
    assert h.exportString() == b""


def test_sparse_string_depends_on_update_order(client, fresh):
    """Registers 4, 3, 2, 1, 0 raised to 1 in that order: Redis' string is VAL(1,1) VAL(1,4)
    XZERO -- the merge scan after the last update cannot join a run of 5 -- where the fewest-bytes
    form of the same registers is VAL(1,4) VAL(1,1) XZERO.  Ascending order gives the latter."""
    rng = np.random.default_rng(62)
    els = _count1_elements(range(5), rng)  # sorted by register
    h = client.getHyperLogLog(fresh)
    h.addAll(Arena(els[::-1]))
    s = h.exportString()
    assert s[16:] == bytes([0x80, 0x83, 0x7F, 0xFA])
    ref = O.RedisHll()
    ref.pfadd(*O.arena(els[::-1]))
    assert s == ref.string(s[8:16])
    g = client.getHyperLogLog(fresh + "a")
    g.addAll(Arena(els))
    assert g.exportString()[16:] == bytes([0x83, 0x80, 0x7F, 0xFA]) == O.hll_sparse_pack(ref.regs)
    h.delete()
    g.delete()


def test_sparse_promotion_at_max_bytes(client, fresh):
    """Promotion to dense inside the PFADD whose element first grows the string past
    hll-sparse-max-bytes (3000), one way; every intermediate GET equals Redis' bytes."""
    rng = np.random.default_rng(12)
    h = client.getHyperLogLog(fresh)
    ref = O.RedisHll()
    crossed = False
    for _ in range(40):
        mat = rng.integers(0, 256, size=(100, 16), dtype=np.uint8)
        assert bool(h.addAll(Arena([bytes(r) for r in mat]))) == bool(ref.pfadd(*O.fixed_arena(mat)))
        s = h.exportString()
        assert s == ref.string(s[8:16])
        crossed = crossed or s[4] == 0
        if crossed:
            assert s[4] == 0 and len(s) == 12304
    assert crossed
    assert h.exportString("dense") == h.exportDense()
    h.delete()


def test_sparse_strings_batched_commands(client, fresh):
    """Multi-key PFADD batches (a key may appear several times: successive rounds) over keys
    that stay sparse, cross the limit mid-command, or start from a SET (non-canonical) string;
    GET bytes equal the Redis restatement after every batch."""
    rng = np.random.default_rng(63)
    keys = [f"{fresh}-{i}" for i in range(6)]
    refs = {k: O.RedisHll() for k in keys}
    # key 5 starts as a SET sparse string with unmerged VALs of one value (Redis keeps it as is)
    raw = bytes([0x84, 0x84, 0x84]) + bytes([0x40 | (16379 >> 8), 16379 & 0xFF]) + bytes([0x80])  # 3 + 16380 + 1
    s5 = _header(1, bytes(7) + b"\x80") + raw
    client.getHyperLogLog(keys[5]).importString(s5)
    refs[keys[5]] = O.RedisHll.from_string(s5)
    for batch in range(6):
        names, els = [], []
        for _ in range(9):
            k = keys[int(rng.integers(0, len(keys)))]
            n = int(rng.integers(0, 3 if k == keys[0] else 600))
            names.append(k)
            els.append(rng.integers(0, 256, size=(n, 16), dtype=np.uint8))
        segs = np.zeros(len(names) + 1, np.uint64)
        segs[1:] = np.cumsum([len(e) for e in els])
        if not segs[-1]:
            continue
        mat = np.concatenate(els)
        replies = hll_add_multi(client, names, segs, Arena.fixed(mat))
        for i, (k, e) in enumerate(zip(names, els)):
            assert bool(replies[i]) == bool(refs[k].pfadd(*O.fixed_arena(e))) or len(e) == 0
        for k in keys:
            h = client.getHyperLogLog(k)
            s = h.exportString()
            if s:
                assert s == refs[k].string(s[8:16]), (batch, k)
    for k in keys:
        client.getHyperLogLog(k).delete()


def test_sparse_merge_write_back_order(client, fresh):
    """PFMERGE into a sparse destination from sparse sources sets the maxima register by
    register, ascending (pfmergeCommand), through hllSparseSet -- runs split and merge as in
    Redis, and the destination promotes if the string outgrows the limit on the way."""
    rng = np.random.default_rng(64)
    d = client.getHyperLogLog(fresh + "d")
    ref = O.RedisHll()
    e0 = rng.integers(0, 256, size=(40, 16), dtype=np.uint8)
    d.addAll(Arena([bytes(x) for x in e0]))
    ref.pfadd(*O.fixed_arena(e0))
    for i, n in enumerate((30, 200, 500, 900)):
        src = client.getHyperLogLog(f"{fresh}s{i}")
        e = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
        src.addAll(Arena([bytes(x) for x in e]))
        r = O.RedisHll()
        r.pfadd(*O.fixed_arena(e))
        d.mergeWith(f"{fresh}s{i}")
        ref.merge_from(np.maximum(ref.regs, r.regs), use_dense=bool(r.dense.value))
        s = d.exportString()
        assert s == ref.string(s[8:16]), i
        src.delete()
    d.delete()


def test_sparse_export_limits_and_merge_encoding(client, fresh):
    regs = O.hll_new()
    regs[[5, 900, 16383]] = [3, 40, 1]  # 40 > 32: only dense can hold it
    big = client.getHyperLogLog(fresh + "big")
    big.importString(_header(0, bytes(7) + b"\x80") + O.hll_dense_pack(regs))
    assert big.exportString()[4] == 0  # SET keeps the imported (dense) encoding
    with pytest.raises(IllegalArgumentException):
        big.exportString("sparse")
    with pytest.raises(IllegalArgumentException):
        big.exportString("rle")
    small = O.hll_new()
    small[[1, 2, 3, 4, 5, 77]] = [2, 2, 2, 2, 2, 32]
    a = client.getHyperLogLog(fresh + "a")
    a.importString(_header(1, bytes(7) + b"\x80") + O.hll_sparse_pack(small))
    b = client.getHyperLogLog(fresh + "b")
    b.add(b"x")
    # all inputs sparse: PFMERGE keeps the destination sparse
    b.mergeWith(fresh + "a")
    m = small.copy()
    O.hll_merge(m, regs_of(b))
    sb = b.exportString()
    assert sb[4] == 1 and np.array_equal(O.hll_sparse_unpack(sb[16:]), m)
    # a dense source makes the destination dense
    b.mergeWith(fresh + "big")
    O.hll_merge(m, regs)
    sb = b.exportString()
    assert sb[4] == 0 and np.array_equal(O.hll_dense_unpack(sb[16:]), m)
    for x in (a, b, big):
        x.delete()


def test_invalid_hll_string(client, fresh):
    with pytest.raises(RedisException):
        client.getHyperLogLog(fresh).importString(b"HYLX" + bytes(12300))
    with pytest.raises(RedisException):
        client.getHyperLogLog(fresh).importString(b"HYLL" + bytes(20))


def test_large_batch_accuracy_and_parity(client, fresh):
    """C4 geometry per HLL (100k 16-byte elements) for 64 HLLs in one PFADD batch."""
    rng = np.random.default_rng(0x5EED0004)
    nh, per = 64, 100_000
    mat = rng.integers(0, 256, size=(nh * per, 16), dtype=np.uint8)
    names = [f"{fresh}-{i}" for i in range(nh)]
    segs = np.arange(nh + 1, dtype=np.uint64) * per
    replies = hll_add_multi(client, names, segs, Arena.fixed(mat))
    assert replies.all()
    counts = hll_count_each(client, names)
    for i in range(0, nh, 8):
        r = O.hll_new()
        O.hll_pfadd(r, *O.fixed_arena(mat[i * per:(i + 1) * per]))
        assert counts[i] == O.hll_count(r)
        assert np.array_equal(regs_of(client.getHyperLogLog(names[i])), r)
    assert np.all(np.abs(counts.astype(np.float64) - per) / per < 0.03)


def _count1_elements(indexes, rng):
    """One 16-byte element per target register index whose MurmurHash64A gives that index and
    count 1 (bit 14 of the hash set: hllPatLen = 1)."""
    want = set(int(i) for i in indexes)
    found = {}
    while len(found) < len(want):
        cand = rng.integers(0, 256, size=(1 << 20, 16), dtype=np.uint8)
        h = O.murmur_batch(*O.fixed_arena(cand))
        idx = (h & np.uint64(16383)).astype(np.int64)
        ok = ((h >> np.uint64(14)) & np.uint64(1)) == 1
        for j in np.nonzero(ok)[0]:
            i = int(idx[j])
            if i in want and i not in found:
                found[i] = bytes(cand[j])
    return [found[i] for i in sorted(want)]


def test_sparse_promotion_is_checked_per_command(client, fresh):
    """Redis promotes during the PFADD that first overflows hll-sparse-max-bytes, even if a later
    PFADD shrinks the sparse form again (merging runs).  Command 1 sets every even register of
    [0, 8000) to 1: 4000 VAL + 4000 ZERO opcodes, > 3000 bytes -> promoted.  Command 2 fills the
    odd ones: the fewest-bytes form of the final registers (2000 VAL opcodes) would fit, but the
    key stays dense (promotion is one way)."""
    rng = np.random.default_rng(61)
    even = _count1_elements(range(0, 8000, 2), rng)
    odd = _count1_elements(range(1, 8000, 2), rng)
    h = client.getHyperLogLog(fresh)
    assert h.addAll(Arena(even))
    assert h.addAll(Arena(odd))
    regs = O.hll_new()
    regs[:8000] = 1
    s = h.exportString()  # as stored
    assert s[4] == 0 and np.array_equal(O.hll_dense_unpack(s[16:]), regs)
    ops = O.hll_sparse_pack(regs)
    assert 16 + len(ops) <= 3000  # what an export-time check would have kept sparse
    h.delete()


def _count_elements(indexes, count, rng):
    """One 16-byte element per register index whose MurmurHash64A gives that index and hllPatLen
    `count` (bits 14 .. 14+count-2 of the hash clear, bit 14+count-1 set)."""
    want = set(int(i) for i in indexes)
    found = {}
    sh = np.uint64(14)
    while len(found) < len(want):
        cand = rng.integers(0, 256, size=(1 << 20, 16), dtype=np.uint8)
        h = O.murmur_batch(*O.fixed_arena(cand))
        idx = (h & np.uint64(16383)).astype(np.int64)
        low = (h >> sh) & np.uint64((1 << count) - 1)
        ok = low == np.uint64(1 << (count - 1))
        for j in np.nonzero(ok)[0]:
            i = int(idx[j])
            if i in want and i not in found:
                found[i] = bytes(cand[j])
    return [found[i] for i in sorted(want)]


def test_sparse_set_string_beyond_limit(client, fresh):
    """A SET sparse string longer than hll-sparse-max-bytes stays sparse through updates that do
    not grow it (VAL of length 1 raised in place), and promotes at the first one that grows it."""
    rng = np.random.default_rng(66)
    ops = bytearray()
    for _ in range(3000):  # registers 0, 2, .., 5998 = 1: 6000 opcode bytes
        ops += bytes([0x80, 0x00])
    rest = 16384 - 6000
    ops += bytes([0x40 | ((rest - 1) >> 8), (rest - 1) & 0xFF])
    s0 = _header(1, bytes(7) + b"\x80") + bytes(ops)
    h = client.getHyperLogLog(fresh)
    h.importString(s0)
    ref = O.RedisHll.from_string(s0)
    raise2 = _count_elements(range(0, 40, 2), 2, rng)  # VAL(1,1) -> VAL(2,1): no growth
    assert h.addAll(Arena(raise2))
    ref.pfadd(*O.arena(raise2))
    s = h.exportString()
    assert s[4] == 1 and len(s) == len(s0) and s == ref.string(s[8:16])
    grow = _count_elements([1], 1, rng)  # ZERO(1) between two VALs -> VAL: no growth either
    h.addAll(Arena(grow))
    ref.pfadd(*O.arena(grow))
    assert h.exportString() == ref.string(h.exportString()[8:16])
    far = _count_elements([9000], 1, rng)  # splits the XZERO: grows past the limit -> dense
    h.addAll(Arena(far))
    ref.pfadd(*O.arena(far))
    s = h.exportString()
    assert s[4] == 0 and s == ref.string(s[8:16])
    h.delete()


def test_sparse_first_batches_many_keys(client, fresh):
    """The sparse-replay shortcut's regime (hll_kernels.hip replay_one, r04): many fresh HLLs in one
    multi-key PFADD, the keys staying sparse (1,000 elements each: their final registers have no
    nonzero run longer than 4, so the string is the normalized encoding), then a second batch into
    the same (normalized) strings, then a third batch that builds runs of five equal registers on
    some keys (the shortcut must not apply: the element-by-element replay decides the split).  GET
    bytes equal the element-by-element restatement for every key after every batch."""
    rng = np.random.default_rng(67)
    nk = 600
    keys = [f"{fresh}-{i}" for i in range(nk)]
    refs = [O.RedisHll() for _ in keys]
    runs5 = _count1_elements(range(5000, 5005), rng)  # registers 5000..5004 raised to 1

    def batch(per, extra=None):
        els = [rng.integers(0, 256, size=(per, 16), dtype=np.uint8) for _ in keys]
        if extra is not None:  # the run of five on every third key, in descending order
            for i in range(0, nk, 3):
                els[i] = np.concatenate([els[i], np.frombuffer(b"".join(extra[::-1]), np.uint8).reshape(-1, 16)])
        segs = np.zeros(nk + 1, np.uint64)
        segs[1:] = np.cumsum([len(e) for e in els])
        replies = hll_add_multi(client, keys, segs, Arena.fixed(np.concatenate(els)))
        for i in range(nk):
            assert bool(replies[i]) == bool(refs[i].pfadd(*O.fixed_arena(els[i])))

    def check(tag):
        sparse = 0
        for k, r in zip(keys, refs):
            s = client.getHyperLogLog(k).exportString()
            assert s == r.string(s[8:16]), (tag, k)
            sparse += s[4] == 1
        return sparse

    batch(1000)
    assert check("first") == nk  # all stay sparse (~2,000 bytes each)
    batch(150)
    assert check("second") == nk
    batch(20, extra=runs5)
    check("third")
    for k in keys:
        client.getHyperLogLog(k).delete()


def test_sparse_set_string_past_the_slot_copies(client, fresh):
    """a pool slot's opcode list holds 3,072 opcodes (a PFADD-built string never exceeds
    the 3,000-byte limit); a SET string with more (here 6,001 opcodes) moves to its own list.  It
    survives a device-to-device copy to another context (rbx_hll_copy_to, the node's cross-GPU
    PFCOUNT / PFMERGE input) byte for byte, and the copy keeps replaying like the original."""
    import ctypes as C

    from redisson_amd import RedissonClient
    from redisson_amd import _lib as L

    rng = np.random.default_rng(68)
    ops = bytearray()
    for _ in range(3000):
        ops += bytes([0x80, 0x00])
    rest = 16384 - 6000
    ops += bytes([0x40 | ((rest - 1) >> 8), (rest - 1) & 0xFF])
    s0 = _header(1, bytes(7) + b"\x80") + bytes(ops)
    client.getHyperLogLog(fresh).importString(s0)
    with RedissonClient(0) as other:
        src, keep1 = L.name_struct(fresh)
        dst, keep2 = L.name_struct(fresh + "-copy")
        assert L.lib().rbx_hll_copy_to(client.ctx, src, other.ctx, dst) == 0
        g = other.getHyperLogLog(fresh + "-copy")
        assert g.exportString() == s0
        raise2 = _count_elements(range(0, 40, 2), 2, rng)  # in place: no growth, stays sparse
        g.addAll(Arena(raise2))
        ref = O.RedisHll.from_string(s0)
        ref.pfadd(*O.arena(raise2))
        s = g.exportString()
        assert s[4] == 1 and s == ref.string(s[8:16])
        g.delete()
    client.getHyperLogLog(fresh).delete()


def test_c4_10k_hlls_three_pool_chunks(client, fresh):
    """config C4 at its HLL count.  10,000 HLLs in ONE multi-key PFADD batch
    (M/RedissonHyperLogLog.java:76-102 addAll per key, pipelined): the register pool holds 4,096
    HLLs per 64 MiB chunk, so the batch spans three chunks.  200..2,400 16-byte elements per key
    (some keys stay sparse, the larger ones promote to dense mid-command).  Checked against the
    oracle: every PFADD reply, every key's PFCOUNT, the GET bytes (sparse or dense as Redis holds
    them) of 150 keys sampled from all three chunks; then pack_registers over all 10,000 (sampled
    rows vs the oracle's registers) and unpack_max of a random register image (every count and
    sampled registers vs max(oracle, image))."""
    import ctypes as C

    import torch

    from redisson_amd import _lib as L

    rng = np.random.default_rng(0xC4C4)
    nk = 10_000
    keys = [f"{fresh}-{i}" for i in range(nk)]
    per = rng.integers(200, 2401, size=nk)
    segs = np.zeros(nk + 1, np.uint64)
    segs[1:] = np.cumsum(per)
    mat = rng.integers(0, 256, size=(int(segs[-1]), 16), dtype=np.uint8)
    replies = hll_add_multi(client, keys, segs, Arena.fixed(mat))
    refs = [O.RedisHll() for _ in keys]
    for i in range(nk):
        ch = refs[i].pfadd(*O.fixed_arena(mat[int(segs[i]):int(segs[i + 1])]))
        assert bool(replies[i]) == bool(ch), i
    counts = hll_count_each(client, keys)
    want = np.array([O.hll_count(r.regs) for r in refs], np.uint64)
    assert np.array_equal(np.asarray(counts, np.uint64), want)
    dense = sum(int(r.dense.value) for r in refs)
    assert 0 < dense < nk  # both encodings occur
    sample = sorted(set(rng.choice(nk, size=147, replace=False).tolist()) | {0, 4095, 4096, 8191, 8192, nk - 1})
    assert any(i < 4096 for i in sample) and any(4096 <= i < 8192 for i in sample) and any(i >= 8192 for i in sample)
    for i in sample:
        s = client.getHyperLogLog(keys[i]).exportString()
        assert s == refs[i].string(s[8:16]), i

    hs = []
    for nm in keys:
        hp = C.c_void_p()
        assert L.lib().rbx_hll_open(client.ctx, nm.encode(), 0, C.byref(hp)) == 0
        hs.append(hp.value)
    arr = (C.c_void_p * nk)(*hs)
    try:
        buf = torch.zeros(nk * 16384, dtype=torch.uint8, device="cuda")
        assert L.lib().rbx_hll_pack_registers(client.ctx, arr, nk, buf.data_ptr(), None) == 0
        L.lib().rbx_synchronize(client.ctx)
        got = buf.view(nk, 16384)
        for i in sample:
            assert np.array_equal(got[i].cpu().numpy(), refs[i].regs), i
        other = torch.randint(0, 4, (nk, 16384), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        assert L.lib().rbx_hll_unpack_max_registers(client.ctx, arr, nk, other.data_ptr(), None) == 0
        out = np.zeros(nk, np.uint64)
        assert L.lib().rbx_hll_count_each_handles(client.ctx, arr, nk, out.ctypes.data_as(L.u64p)) == 0
        oth = other.cpu().numpy()
        mx = np.maximum(np.stack([r.regs for r in refs]), oth)
        want2 = np.array([O.hll_count(mx[i]) for i in range(nk)], np.uint64)
        assert np.array_equal(out, want2)
        for i in sample:
            d = client.getHyperLogLog(keys[i]).exportDense()
            assert np.array_equal(O.hll_dense_unpack(d[16:]), mx[i]), i
    finally:
        for h in hs:
            L.lib().rbx_hll_close(h)
    for nm in keys:
        client.getHyperLogLog(nm).delete()


def _shortcut_case(kind, rng):
    """Element lists (16-byte, count-1 or count-2 elements at chosen registers) for the boundaries of
    the normalized-string shortcut (hll_kernels.hip replay_one): the shortcut applies when
    the final registers have no nonzero run longer than 4 and 16 + B <= 3000 (B = bytes of the maximal
    zero runs + one byte per nonzero register)."""
    if kind == "runs_of_exactly_4":
        # registers 100..103 -> 1 and 300..303 -> 2: runs of exactly four equal registers
        els = _count1_elements(range(100, 104), rng) + _count_elements(range(300, 304), 2, rng)
        els += _count1_elements(rng.choice(np.arange(1000, 16000), size=200, replace=False), rng)
    elif kind == "B_exactly_2984":
        # registers 1, 3, ..., 2981 -> 1: B = 1491 VALs + 1491 ZERO(1) + a 2-byte XZERO = 2984
        els = _count1_elements(range(1, 2982, 2), rng)
    elif kind == "B_2985_promotes":
        # one nonzero register more (2983): 16 + B = 3002, and no encoding of the registers is shorter
        els = _count1_elements(range(1, 2984, 2), rng)
    elif kind == "pairs_past_B_within_fewest":
        # registers 3i, 3i+1 -> 1 for i < 1000: B = 3002 (shortcut off), the fewest-bytes encoding (VAL(1,2)
        # per pair) ~2002: neither shortcut decides, the element-by-element replay does
        idx = np.sort(np.concatenate([np.arange(0, 3000, 3), np.arange(1, 3000, 3)]))
        els = _count1_elements(idx, rng)
    else:
        raise AssertionError(kind)
    order = rng.permutation(len(els))
    return [els[int(i)] for i in order]


@pytest.mark.parametrize("kind", ["runs_of_exactly_4", "B_exactly_2984", "B_2985_promotes",
                                  "pairs_past_B_within_fewest"])
def test_sparse_shortcut_boundaries(client, fresh, kind):
    """byte-level checks at the boundaries of the sparse-replay shortcut -- runs of exactly
    four equal registers, B exactly at the limit (16 + B = 3000) and one register past it, and strings
    whose B is past the limit while their fewest-bytes encoding fits (element-by-element replay).  One
    PFADD per key, elements in random order; the GET bytes equal the hllSparseSet restatement
    (oracle RedisHll; Redis's hyperloglog.c itself is not in the reference: parity with a live Redis
    stays unpinned)."""
    rng = np.random.default_rng(abs(hash(kind)) % (1 << 32))
    els = _shortcut_case(kind, rng)
    h = client.getHyperLogLog(fresh)
    assert h.addAll(Arena(els)) is True
    ref = O.RedisHll()
    ref.pfadd(*O.arena(els))
    s = h.exportString()
    assert s == ref.string(s[8:16])
    if kind == "B_exactly_2984":
        assert s[4] == 1 and len(s) == 3000
    if kind == "B_2985_promotes":
        assert s[4] == 0
    h.delete()


@pytest.mark.parametrize("lead", [0, 1])
def test_sparse_set_string_just_under_the_limit(client, fresh, lead):
    """a SET (imported) sparse string of 2,999 / 3,000 bytes (normalized: 1,491 VAL(1,1) with a
    ZERO(1) between neighbours from register `lead`, a leading ZERO(1) when lead = 1, then one XZERO),
    then PFADDs that raise VALs in place (no growth), fill ZERO(1)s between VALs of another value (no
    growth) and split the XZERO (growth past the limit -> dense)."""
    rng = np.random.default_rng(400 + lead)
    regs = O.hll_new()
    regs[lead:lead + 2 * 1491:2] = 1
    ops = _sparse_encode(regs)
    s0 = _header(1, bytes(7) + b"\x80") + ops
    assert len(s0) == 2999 + lead
    h = client.getHyperLogLog(fresh)
    h.importString(s0)
    ref = O.RedisHll.from_string(s0)
    for batch in (_count_elements([lead, lead + 2, lead + 4], 2, rng), _count1_elements([lead + 1, lead + 3], rng),
                  _count1_elements([12000], rng)):
        h.addAll(Arena(batch))
        ref.pfadd(*O.arena(batch))
        s = h.exportString()
        assert s == ref.string(s[8:16])
    assert s[4] == 0  # the split of the XZERO grew the string past the limit
    h.delete()
