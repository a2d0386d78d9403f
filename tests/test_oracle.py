"""Pins the CPU oracle (oracle/rbx_oracle.c) and cross-checks it against the independent
pure-Python restatement (oracle/pyref.py).  CPU only."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import pyref as P

# Upstream google/highwayhash test vectors: key {0x0706050403020100, ...}, input bytes
# 0,1,...,len-1 (highwayhash/highwayhash_test.cc kExpected64 / kExpected128).  Redisson's
# HighwayHash.java is the upstream portable Java implementation (finalize128 included).
KAT_KEY = [0x0706050403020100, 0x0F0E0D0C0B0A0908, 0x1716151413121110, 0x1F1E1D1C1B1A1918]
KAT64 = [0x907A56DE22C26E53, 0x7EAB43AAC7CDDD78, 0xB8D0569AB0B53D62, 0x5C6BEFAB8A463D80,
         0xF205A46893007EDA, 0x2B8A1668E4A94541, 0xBD4CCC325BEFCA6F, 0x4D02AE1738F59482,
         0xE1205108E55F3171, 0x32D2644EC77A1584, 0xF6E10ACDB103A90B, 0xC3BBF4615B415C15]
KAT128 = [(0x0FED268F9D8FFEC7, 0x33565E767F093E6F), (0xD6B0A8893681E7A8, 0xDC291DF9EB9CDCB4),
          (0x3D15AD265A16DA04, 0x78085638DC32E868)]


@pytest.mark.parametrize("n", range(len(KAT64)))
def test_highwayhash64_kat(n):
    d = bytes(range(n))
    assert O.highway_hash64(d, KAT_KEY) == KAT64[n]
    assert P.highway_hash64(d, KAT_KEY) == KAT64[n]


@pytest.mark.parametrize("n", range(len(KAT128)))
def test_highwayhash128_kat(n):
    d = bytes(range(n))
    assert O.highway_hash128(d, KAT_KEY) == KAT128[n]


def test_hash128_c_vs_python_all_tail_shapes():
    rng = np.random.default_rng(1)
    for L in range(0, 130):
        d = rng.bytes(L)
        assert O.redisson_hash128(d) == P.highway_hash128(d), L


def test_murmur64a_smhasher_verification():
    # SMHasher VerificationTest: keys {0..i-1} hashed with seed 256-i, then the 256
    # 8-byte hashes hashed with seed 0; low 32 bits == 0x1F0D3804 for MurmurHash64A.
    key = bytearray(256)
    hashes = bytearray()
    for i in range(256):
        key[i] = i
        hashes += O.murmur64a(bytes(key[:i]), 256 - i).to_bytes(8, "little")
    assert O.murmur64a(bytes(hashes), 0) & 0xFFFFFFFF == 0x1F0D3804


def test_murmur_c_vs_python():
    rng = np.random.default_rng(2)
    for L in range(0, 70):
        d = rng.bytes(L)
        assert O.murmur64a(d) == P.murmur64a(d)
        assert O.hll_patlen(d) == P.hll_patlen(d)


def test_crc16_kat_and_slots():
    assert O.crc16(b"123456789") == 0x31C3  # Redis Cluster spec
    assert P.crc16(b"123456789") == 0x31C3
    for k in [b"foo{bar}baz", b"{user1000}.following", b"{}", b"a}b{c}", b"x{}y", b"{a", b""]:
        assert O.calc_slot(k) == P.calc_slot(k)
    assert O.calc_slot(b"{user1000}.following") == O.calc_slot(b"{user1000}.followers")


def test_bloom_config_kat():
    # T/RedissonBloomFilterTest.java:69-76
    assert O.bloom_optimal(100, 0.03) == (729, 5)
    # BASELINE.md derived parameters
    assert O.bloom_optimal(10_000_000, 0.01) == (95850583, 7)
    assert O.bloom_optimal(1_000_000, 1e-3) == (14377587, 10)
    assert O.bloom_optimal(448_089_842, 0.01) == (4294967293, 7)


@pytest.mark.parametrize("n,p", [(1, -1), (1, 2), (1, 1), (10**12, 1e-9)])
def test_bloom_config_illegal_argument(n, p):
    # testFalseProbability1/2, testSizeZero (:44-66); size > getMaxSize()
    with pytest.raises(O.OracleError):
        O.bloom_optimal(n, p)


def test_bloom_indexes_python_vs_c():
    rng = np.random.default_rng(3)
    for _ in range(200):
        h1, h2 = int(rng.integers(0, 2**63)) * 2 + 1, int(rng.integers(0, 2**63))
        for size, k in [(729, 5), (95850583, 7), (2**32, 7), (4294967293, 40)]:
            assert O.bloom_indexes(h1, h2, k, size) == P.bloom_indexes(h1, h2, k, size)


def test_wide_size_offset_limit():
    """|size| > 2^32 (tryInit with a negative expectedInsertions): a SETBIT / GETBIT past the Redis
    offset limit 2^32 - 1 is an error reply; the batch's other SETBITs still run and the call then
    throws (RedisException, -9).  Checked key by key against pyref's indexes."""
    size, k = O.bloom_optimal(-500_000_000, 0.01)
    assert size < -(1 << 32) and k == 7
    rng = np.random.default_rng(17)
    f = O.OracleBloom(size, k)
    expect_bits, n_ok, n_err = set(), 0, 0
    for i in range(64):
        key = rng.bytes(16)
        h1, h2 = P.highway_hash128(key)
        idx = P.bloom_indexes(h1, h2, k, size)
        oob = any(x > 0xFFFFFFFF for x in idx)
        new = any(x <= 0xFFFFFFFF and x not in expect_bits for x in idx)
        c = f.add(*O.arena([key]))
        expect_bits.update(x for x in idx if x <= 0xFFFFFFFF)
        if oob:
            assert c == -9
            n_err += 1
        else:
            assert c == int(new)
            n_ok += 1
        assert f.contains(*O.arena([key])) == (-9 if oob else 1)
    assert n_ok > 5 and n_err > 5  # P(no index past the limit) = (2^32 / |size|)^7 ~ 0.46
    bits = np.unpackbits(f.bitmap[: f.redis_len])
    assert set(np.flatnonzero(bits).tolist()) == expect_bits
    assert f.redis_len == max(expect_bits) // 8 + 1


def test_java_math_round():
    assert O.java_math_round(0.49999999999999994) == 0
    assert O.java_math_round(0.5) == 1
    assert O.java_math_round(-0.5) == 0
    assert O.java_math_round(-1.5) == -1
    assert O.java_math_round(2.5) == 3
    assert O.java_math_round(float("inf")) == 2**63 - 1
    assert O.java_math_round(float("nan")) == 0


def _sk(xs):
    return O.arena([x.encode() for x in xs])


def test_redisson_bloom_tests_replay_on_oracle():
    # T/RedissonBloomFilterTest.java testContainsAll / testAddAll, StringCodec bytes
    f = O.OracleBloom(*O.bloom_optimal(100, 0.03))
    assert f.contains(*_sk(["1", "2", "3"])) == 0
    assert f.add(*_sk(["1", "2", "3"])) == 3
    assert f.contains(*_sk(["1", "2", "3"])) == 3
    assert f.contains(*_sk(["1", "5"])) == 1
    g = O.OracleBloom(*O.bloom_optimal(100, 0.03))
    assert g.add(*_sk(["1", "2", "3"])) == 3
    assert g.add(*_sk(["1", "2", "3"])) == 0
    assert g.count() == 3
    assert g.add(*_sk(["1", "5"])) == 1
    assert g.count() == 4


def test_empty_collection_is_arithmetic_exception():
    f = O.OracleBloom(729, 5)
    assert f.add(*O.arena([])) == -4
    assert f.contains(*O.arena([])) == -4


def test_hll_reference_counts():
    # T/RedissonHyperLogLogTest.java and the Redis PFADD/PFCOUNT/PFMERGE doc examples
    def pf(regs, xs):
        return O.hll_pfadd(regs, *_sk(xs))

    r = O.hll_new()
    pf(r, ["1", "2", "3"])
    assert O.hll_count(r) == 3
    h1, h2 = O.hll_new(), O.hll_new()
    assert [pf(h1, [x]) for x in ["foo", "bar", "zap", "a"]] == [1, 1, 1, 1]
    assert [pf(h2, [x]) for x in ["a", "b", "c", "foo", "c"]] == [1, 1, 1, 1, 0]
    h3 = O.hll_new()
    O.hll_merge(h3, h1)
    O.hll_merge(h3, h2)
    assert O.hll_count(h3) == 6
    h = O.hll_new()
    pf(h, ["1", "2", "3", "4", "5"])
    assert O.hll_count(h) == 5
    pf(h, ["6", "7", "8", "8", "9", "10"])
    assert O.hll_count(h) == 10
    assert O.hll_count(O.hll_new()) == 0


def test_hll_dense_pack_roundtrip():
    rng = np.random.default_rng(5)
    regs = rng.integers(0, 64, size=16384, dtype=np.uint8)
    assert np.array_equal(O.hll_dense_unpack(O.hll_dense_pack(regs)), regs)


def test_hll_estimator_accuracy():
    rng = np.random.default_rng(6)
    for n in (1000, 100000):
        regs = O.hll_new()
        O.hll_pfadd(regs, *O.fixed_arena(rng.integers(0, 256, size=(n, 16), dtype=np.uint8)))
        assert abs(O.hll_count(regs) - n) / n < 0.03


def test_hll_sparse_pack_opcodes():
    # [redis-7.2] hyperloglog.c opcodes: an empty HLL is one XZERO of 16384 registers
    assert O.hll_sparse_pack(O.hll_new()) == b"\x7f\xff"
    regs = O.hll_new()
    regs[0:5] = 3        # VAL(3) x4 + VAL(3) x1
    regs[69] = 32        # ZERO run of 64, VAL(32) x1, then XZERO of the rest
    assert O.hll_sparse_pack(regs) == bytes([0x8B, 0x88, 0x3F, 0xFC, 0x40 | (16313 >> 8), 16313 & 0xFF])
    regs[70] = 33
    assert O.hll_sparse_pack(regs) is None
    rng = np.random.default_rng(7)
    for fill in (0.01, 0.2, 1.0):
        r = np.where(rng.random(16384) < fill, rng.integers(1, 33, 16384), 0).astype(np.uint8)
        assert np.array_equal(O.hll_sparse_unpack(O.hll_sparse_pack(r)), r)


def _sp_set(ops, n, index, count, max_bytes=3000):
    import ctypes as C
    ln = C.c_size_t(n)
    r = O.lib().orc_hll_sparse_set(O._p(ops), C.byref(ln), ops.size, index, count, max_bytes)
    return r, ln.value


def test_hll_sparse_set_known_answers():
    """hllSparseSet restatement [redis-7.2 hyperloglog.c, external; parity unpinned: no live
    redis-server here] on hand-derived cases: case D splits of XZERO / ZERO / VAL, cases A-C,
    the VAL merge scan, promotion on count > 32 and on hll-sparse-max-bytes."""
    def fresh():
        ops = np.zeros(20000, np.uint8)
        return ops, O.lib().orc_hll_sparse_new(O._p(ops))

    ops, n = fresh()
    assert ops[:n].tobytes() == b"\x7f\xff"
    r, n = _sp_set(ops, n, 100, 3)  # XZERO -> XZERO(100) VAL(3,1) XZERO(16283)
    assert r == 1 and ops[:n].tobytes() == bytes([0x40, 99, 0x88, 0x40 | (16282 >> 8), 16282 & 0xFF])
    r, n = _sp_set(ops, n, 10, 1)  # XZERO(100) -> ZERO(10) VAL(1,1) XZERO(89): 89 > 64
    assert r == 1 and ops[:5].tobytes() == bytes([9, 0x80, 0x40, 88, 0x88])
    assert _sp_set(ops, n, 100, 2) == (0, n)  # case A: VAL 3 >= 2
    r, n = _sp_set(ops, n, 100, 5)  # case B: VAL len 1 raised in place
    assert r == 1 and ops[4] == 0x80 | (4 << 2)
    assert _sp_set(ops, n, 7, 33)[0] == 2  # count > 32: promote
    # descending 4..0 -> VAL(1,1) VAL(1,4) XZERO; ascending -> VAL(1,4) VAL(1,1) XZERO
    ops, n = fresh()
    for i in (4, 3, 2, 1, 0):
        r, n = _sp_set(ops, n, i, 1)
    assert ops[:n].tobytes() == bytes([0x80, 0x83, 0x7F, 0xFA])
    ops, n = fresh()
    for i in (0, 1, 2, 3, 4):
        r, n = _sp_set(ops, n, i, 1)
    assert ops[:n].tobytes() == bytes([0x83, 0x80, 0x7F, 0xFA])
    # VAL split: VAL(2,4) at 0..3, raise register 1 -> VAL(2,1) VAL(5,1) VAL(2,2)
    ops, n = fresh()
    for i in range(4):
        r, n = _sp_set(ops, n, i, 2)
    assert ops[:n].tobytes() == bytes([0x87, 0x7F, 0xFB])
    r, n = _sp_set(ops, n, 1, 5)
    assert ops[:n].tobytes() == bytes([0x84, 0x90, 0x85, 0x7F, 0xFB])
    # the size limit: every even register set costs 2 bytes; the update that would pass 3000
    # returns 2 and leaves the string as it was
    ops, n = fresh()
    j = 0
    while True:
        before = ops[:n].tobytes()
        r, n2 = _sp_set(ops, n, j, 1)
        if r == 2:
            assert n2 == n and ops[:n].tobytes() == before and 16 + n + 2 > 3000
            break
        assert r == 1 and 16 + n2 <= 3000
        n, j = n2, j + 2
    assert j > 1000


def test_redis_hll_model_invariants():
    """RedisHll (PFADD element by element): while sparse the string decodes to the registers and
    fits hll-sparse-max-bytes; the registers equal the order-free PFADD; promotion is one way."""
    rng = np.random.default_rng(65)
    h = O.RedisHll()
    regs = O.hll_new()
    was_dense = False
    for _ in range(30):
        e = rng.integers(0, 256, size=(int(rng.integers(1, 150)), 16), dtype=np.uint8)
        h.pfadd(*O.fixed_arena(e))
        O.hll_pfadd(regs, *O.fixed_arena(e))
        assert np.array_equal(h.regs, regs)
        if h.dense.value:
            was_dense = True
        else:
            assert not was_dense
            assert np.array_equal(O.hll_sparse_unpack(h.sparse_ops), regs) and 16 + h.len.value <= 3000
    assert was_dense


def test_multithreaded_restatement_matches_single_thread():
    """rbx_oracle_mt.c (bench.py's all-core cpu_baseline) == rbx_oracle.c, per key and bitmap."""
    rng = np.random.default_rng(31)
    for size, k, n in [(9585, 7, 3000), (95_850_583, 7, 200_000), (-2000, 5, 1500), (64, 3, 500)]:
        keys = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
        keys[n // 3: n // 3 + 50] = keys[:50]  # duplicates: only the first copy is new
        a, b = O.OracleBloom(size, k), O.OracleBloom(size, k)
        c1, f1 = a.add(*O.fixed_arena(keys), per_key=True)
        c2, f2 = b.add_mt(*O.fixed_arena(keys), nthreads=7, per_key=True)
        assert c1 == c2 and np.array_equal(f1, f2), (size, k)
        assert a.redis_len == b.redis_len and a.redis_string() == b.redis_string()
        probe = np.concatenate([keys[: n // 2], rng.integers(0, 256, size=(n, 16), dtype=np.uint8)])
        r1 = a.contains(*O.fixed_arena(probe), per_key=True)
        r2 = b.contains_mt(*O.fixed_arena(probe), nthreads=5, per_key=True)
        assert r1[0] == r2[0] and np.array_equal(r1[1], r2[1])


def test_stream_restatement_matches_per_key_batches():
    """orc_bloom_stream (the C5 checker) == one add(T)/contains(T) batch per command, in order."""
    rng = np.random.default_rng(1)
    shapes = [(64, 7), (729, 5), (9585, 7), (-2000, 3)]
    a = [O.OracleBloom(m, k) for m, k in shapes]
    b = [O.OracleBloom(m, k) for m, k in shapes]
    n = 4000
    keys = rng.integers(0, 256, size=(n // 3, 16), dtype=np.uint8)[rng.integers(0, n // 3, size=n)]
    kf = rng.integers(0, len(shapes), size=n).astype(np.uint32)
    op = (rng.random(n) < 0.4).astype(np.uint8)
    out, cnt = O.bloom_stream(a, kf, op, keys, None, stride=16)
    want = np.array([(b[f].add if o else b[f].contains)(*O.fixed_arena(keys[i:i + 1]))
                     for i, (f, o) in enumerate(zip(kf, op))], np.uint8)
    assert np.array_equal(out, want)
    assert cnt == [int(want[op == 0].sum()), int(want[op == 1].sum())]
    assert all(x.redis_string() == y.redis_string() for x, y in zip(a, b))
    # the arena form (variable-length keys) agrees with the fixed-stride form
    c = [O.OracleBloom(m, k) for m, k in shapes]
    out2, cnt2 = O.bloom_stream(c, kf, op, *O.fixed_arena(keys))
    assert np.array_equal(out2, out) and cnt2 == cnt


from bitset_vectors import BITSET_VECTORS, key_for_bit  # noqa: E402


@pytest.mark.parametrize("bits,size_bits,card", BITSET_VECTORS)
def test_bitset_vectors_on_oracle(bits, size_bits, card):
    f = O.OracleBloom(64, 1)
    keys = [key_for_bit(b) for b in bits]
    assert f.add(*O.arena(keys)) == len(bits)  # every SETBIT returned 0 (testSetGet: set() is false)
    assert f.redis_len * 8 == size_bits and f.bitcount() == card
    s = f.redis_string()
    got = [i for i in range(len(s) * 8) if s[i >> 3] & (0x80 >> (i & 7))]
    assert got == sorted(bits)  # MSB-first: bit i is byte i >> 3, mask 0x80 >> (i & 7)
    assert f.contains(*O.arena([key_for_bit(0)])) == (1 if 0 in bits else 0)  # get(0) is false


def _normalized_bound(regs):
    """(no nonzero run longer than 4, B = zero-run bytes + one byte per nonzero register)."""
    r = np.asarray(regs)
    edges = np.flatnonzero(np.diff(r.astype(np.int16))) + 1
    starts = np.concatenate([[0], edges])
    ends = np.concatenate([edges, [16384]])
    lens, vals = ends - starts, r[starts]
    zero = vals == 0
    b = int(np.where(lens[zero] > 64, 2, 1).sum() + lens[~zero].sum())
    return bool((lens[~zero] <= 4).all()), b


@pytest.mark.parametrize("seed", range(2))
def test_sparse_normalized_shortcut(seed):
    """The property k_hll_sparse_replay's shortcut rests on (hll_kernels.hip replay_one): starting
    from a normalized sparse string (== hll_sparse_pack of its registers, every nonzero run <= 4),
    ANY order of hllSparseSet updates whose final registers have no nonzero run longer than 4 and
    whose bound B (zero-run bytes + one byte per nonzero register) fits hll-sparse-max-bytes ends,
    without a promotion, in hll_sparse_pack of the final registers.  Checked against the
    element-by-element restatement on random windows (clustered registers, few values, repeated
    raises, both ends of the register space) -- the cases where the order could matter."""
    rng = np.random.default_rng(1000 + seed)
    tested = 0
    for _ in range(1000):
        W = int(rng.choice([int(rng.integers(2, 13)), int(rng.integers(2, 13)), 40, 400, 16384]))
        base = int(rng.choice([0, 16384 - W, int(rng.integers(0, 16384 - W + 1))]))
        maxv = int(rng.choice([1, 2, 3, 32]))
        regs = np.zeros(16384, np.uint8)
        nv = int(rng.integers(0, W))
        if nv and rng.random() < 0.7:
            regs[rng.integers(base, base + W, size=nv)] = rng.integers(1, maxv + 1, size=nv)
        ok0, _ = _normalized_bound(regs)
        if not ok0:
            continue
        s0 = O.hll_sparse_pack(regs)
        ops = np.zeros(20000, np.uint8)
        ops[:len(s0)] = np.frombuffer(s0, np.uint8)
        n = len(s0)
        nu = int(rng.integers(1, 2 * min(W, 400) + 4))
        ur, uc = rng.integers(base, base + W, size=nu), rng.integers(1, maxv + 1, size=nu)
        fin = regs.copy()
        np.maximum.at(fin, ur, uc.astype(np.uint8))
        ok, b = _normalized_bound(fin)
        if not ok or 16 + b > 3000:
            continue
        for r_, c_ in zip(ur, uc):
            res, n = _sp_set(ops, n, int(r_), int(c_))
            assert res != 2, "promotion below the B bound"
        assert ops[:n].tobytes() == O.hll_sparse_pack(fin)
        tested += 1
    assert tested > 500
