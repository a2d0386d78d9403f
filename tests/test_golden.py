"""The oracle reproduces the committed golden fixtures (tests/golden/golden.json)."""
import base64
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
SEED = 0x5EED0000


def hll_elements(n):
    return np.random.default_rng(SEED + 4 * 1000003 + n).integers(0, 256, size=(n, 16), dtype=np.uint8)


def test_hash128_fixture():
    for e in G["hash128"]:
        h1, h2 = O.redisson_hash128(bytes.fromhex(e["data"]))
        assert (f"{h1:016x}", f"{h2:016x}") == (e["h1"], e["h2"])


def test_bloom_index_fixture():
    ks = [bytes.fromhex(x) for x in G["bloom_index_keys"]]
    b, o = O.arena(ks)
    for name, c in G["bloom_indexes"].items():
        assert O.bloom_hash_batch(b, o, c["k"], c["size"]).tolist() == c["indexes"], name


def test_bloom_sequence_fixture():
    for s in G["bloom_sequences"]:
        f = O.OracleBloom(s["size"], s["k"])
        for b in s["batches"]:
            c, flags = f.add(*O.arena([bytes.fromhex(x) for x in b["keys"]]), per_key=True)
            assert c == b["count"] and flags.tolist() == b["new"]
        c, pres = f.contains(*O.arena([bytes.fromhex(x) for x in s["probes"]]), per_key=True)
        assert c == s["contains"] and pres.tolist() == s["present"]
        assert f.redis_string().hex() == s["bitmap"] and f.redis_len == s["redis_len"]
        assert f.count() == s["count"]


def test_murmur_fixture():
    for e in G["murmur"]:
        d = bytes.fromhex(e["e"])
        assert f"{O.murmur64a(d):016x}" == e["h"]
        assert list(O.hll_patlen(d)) == [e["reg"], e["count"]]


@pytest.mark.parametrize("i", range(8))
def test_hll_fixture(i):
    e = G["hll"][i]
    regs = O.hll_new()
    if e["n"]:
        O.hll_pfadd(regs, *O.fixed_arena(hll_elements(e["n"])))
    assert base64.b64encode(O.hll_dense_pack(regs)).decode() == e["dense"]
    assert O.hll_count(regs) == e["count"]


def test_slot_fixture():
    for e in G["slots"]:
        assert O.crc16(e["key"].encode()) == e["crc16"]
        assert O.calc_slot(e["key"].encode()) == e["slot"]
