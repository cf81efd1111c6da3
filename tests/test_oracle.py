"""Pin the CPU oracle (test infrastructure) before trusting it.

Pins available offline: the GF(2^8)/generator checks and
KATs of SURVEY Appendix A/B (restated from zfec's published fec.c), two
independent generator derivations, the MDS property, and the semantics of
the reference's own tests (crates/storb_base/src/piece.rs:506-689). Parity
bytes are NOT pinned by any zfec-rs output ("parity unpinned").
"""
import hashlib
import itertools
import json
import os
import random

import numpy as np
import pytest

from oracle import coracle as co
from oracle import zfec_np as zn

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "zfec_vectors.json")


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


# ----------------------------------------------------------- Appendix A.1
def test_gf_tables_appendix_a1():
    L = co.lib()
    assert [L.zo_gf_exp(i) for i in range(10)] == [1, 2, 4, 8, 16, 32, 64, 128, 29, 58]
    assert L.zo_gf_mul(2, 0x80) == 0x1D
    assert L.zo_gf_mul(0x53, 0xCA) == 0x8F
    assert L.zo_gf_inv(2) == 0x8E
    for a in range(1, 256):
        assert L.zo_gf_mul(a, L.zo_gf_inv(a)) == 1
    # numpy twin agrees on the whole multiplication table
    for a in range(256):
        assert all(L.zo_gf_mul(a, b) == zn.GF_MUL[a, b] for b in range(0, 256, 17))


# ----------------------------------------------------------- Appendix A.2/B
APPENDIX_B_ROWS = {
    (4, 6): ["7740380e", "c7a70d6c"],
    (8, 12): ["8918d07d92a4f5fe", "36f8d0ce2519fb16", "5fcda3405048f69e", "ed912490dc9057d2"],
    (2, 3): ["0302"],
    (1, 2): ["01"],
}


@pytest.mark.parametrize("kn", list(APPENDIX_B_ROWS))
def test_generator_rows_appendix_b(kn):
    k, n = kn
    got = [bytes(r).hex() for r in co.enc_matrix(k, n)[k:]]
    assert got == APPENDIX_B_ROWS[kn]


def test_generator_three_derivations_agree():
    for k, n in [(1, 2), (2, 3), (3, 5), (4, 6), (5, 8), (6, 9), (8, 12), (16, 24),
                 (20, 30), (32, 48), (1, 256), (100, 120)]:
        c = co.enc_matrix(k, n)
        assert (c == zn.enc_matrix_gauss(k, n)).all(), (k, n)
        if k <= 32:
            assert (c == zn.enc_matrix_lagrange(k, n)).all(), (k, n)
        assert (c[:k] == np.eye(k, dtype=np.uint8)).all()


def test_generator_rows_xor_to_one():
    # Lagrange basis sums to 1 => constant data gives constant parity.
    for k, n in [(2, 3), (4, 6), (8, 12), (16, 24), (32, 48), (7, 19)]:
        enc = co.enc_matrix(k, n)
        for r in enc[k:]:
            assert np.bitwise_xor.reduce(r) == 1


def test_invalid_params_rejected():
    for k, n in [(0, 2), (3, 2), (2, 257), (0, 0)]:
        with pytest.raises(ValueError):
            co.enc_matrix(k, n)
    with pytest.raises(ValueError):
        co.encode(4, 6, b"")


APPENDIX_B_KATS = [
    (4, 6, "01020304", ["87", "2e"]),
    (4, 6, "00010203040506070809", ["2ec26e", "f142fa"]),
    (4, 6, "ffffffff", ["ff", "ff"]),
    (8, 12, "0102030405060708", ["70", "25", "e1", "6e"]),
    (2, 3, b"Test data".hex(), ["346d7d5e60"]),
    (1, 2, b"Hello, World!".hex(), [b"Hello, World!".hex()]),
]


@pytest.mark.parametrize("k,n,data,parity", APPENDIX_B_KATS)
def test_kats_appendix_b(k, n, data, parity):
    shares, B, pad = co.encode(k, n, bytes.fromhex(data))
    assert [bytes(s).hex() for s in shares[k:]] == parity
    assert B * k - pad == len(bytes.fromhex(data))


def test_k1_parity_is_a_copy():
    d = co.splitmix_bytes(3, 777)
    shares, _, _ = co.encode(1, 4, d)
    for s in shares:
        assert np.array_equal(s, d)


# ----------------------------------------------------------- fixtures
def _data(v):
    if "seed" in v:
        return co.splitmix_bytes(v["seed"], v["len"])
    return np.frombuffer(bytes.fromhex(v["data_hex"]), dtype=np.uint8)


def test_c_oracle_reproduces_golden_vectors(golden):
    for v in golden["kats"] + golden["vectors"] + golden["reference_tests"]:
        k, n = v["k"], v["n"]
        d = _data(v)
        shares, B, pad = co.encode(k, n, d)
        assert (B, pad) == (v["B"], v["padlen"])
        assert [sha(s) for s in shares[k:]] == v["parity_sha256"]
        if "parity_hex" in v:
            assert [bytes(s).hex() for s in shares[k:]] == v["parity_hex"]
        surv = v["decode"]["survivors"]
        rec = co.decode(k, n, [shares[i] for i in surv], surv, B, pad)
        assert sha(rec) == v["decode"]["data_sha256"]


def test_golden_generators(golden):
    for key, rows in golden["generator"].items():
        k, n = map(int, key.split(","))
        assert [bytes(r).hex() for r in co.enc_matrix(k, n)[k:]] == rows


def test_golden_sizing(golden):
    for L, pl, k, m in golden["sizing"]:
        assert co.piece_length(L) == pl
        assert co.get_k_and_m(L) == (k, m)


# ----------------------------------------------------------- MDS / decode
@pytest.mark.parametrize("k,n", [(1, 2), (2, 3), (3, 5), (4, 6), (6, 9), (8, 12)])
def test_every_k_subset_decodes(k, n):
    d = co.splitmix_bytes(k * 100 + n, k * 50 + 3)
    shares, B, pad = co.encode(k, n, d)
    for sub in itertools.combinations(range(n), k):
        assert co.decode(k, n, [shares[i] for i in sub], sub, B, pad) == d.tobytes()


def test_decode_uses_first_k_by_index():
    # piece.rs:368-381 sorts by piece_idx and keeps the first k: a corrupt
    # share beyond the first k must not matter.
    k, n = 4, 6
    d = co.splitmix_bytes(11, 4000)
    shares, B, pad = co.encode(k, n, d)
    bad = [s.copy() for s in shares]
    bad[5][:] ^= 0xFF
    order = [5, 3, 1, 4, 2]  # first 4 by index: 1,2,3,4
    assert co.decode(k, n, [bad[i] for i in order], order, B, pad) == d.tobytes()


def test_decode_errors():
    k, n = 4, 6
    shares, B, pad = co.encode(k, n, co.splitmix_bytes(1, 100))
    with pytest.raises(ValueError):
        co.decode(k, n, shares[:3], [0, 1, 2], B, pad)
    with pytest.raises(ValueError):
        co.decode(k, n, [shares[0], shares[0], shares[1], shares[2]], [0, 0, 1, 2], B, pad)
    with pytest.raises(ValueError):
        co.decode(k, n, shares[:4], [0, 1, 2, 9], B, pad)


def test_numpy_twin_matches_c_oracle_random():
    rng = random.Random(9)
    for _ in range(40):
        k = rng.randrange(1, 20)
        n = rng.randrange(k, k + 12)
        L = rng.randrange(1, 5000)
        d = co.splitmix_bytes(rng.randrange(1 << 40), L)
        a, B, p = co.encode(k, n, d)
        b, B2, p2 = zn.encode(k, n, d)
        assert (B, p) == (B2, p2) and np.array_equal(a, b)
        surv = rng.sample(range(n), k)
        assert zn.decode(k, n, [a[i] for i in surv], surv, p) == d.tobytes()


# ----------------------------------------------------------- sizing
def test_piece_length_reference_test():
    # piece.rs:506-510
    assert co.piece_length(1000) >= 16 * 1024
    assert co.piece_length(1000000) <= 256 * 1024 * 1024


def test_piece_length_table_appendix_a5():
    table = {256 << 10: (2, 3), 512 << 10: (4, 6), 1 << 20: (4, 6), 2 << 20: (8, 12),
             4 << 20: (8, 12), 8 << 20: (16, 24), 16 << 20: (16, 24), 32 << 20: (32, 48),
             1000: (1, 2), 16383: (1, 2), 3 << 20: (6, 9)}
    for L, km in table.items():
        assert co.get_k_and_m(L) == km, L
    assert co.piece_length(0) == 16 * 1024  # release-mode masked shift
    assert co.piece_length(1 << 62) == 256 << 20
    assert co.piece_length(4 << 20) == 512 << 10
    assert co.piece_length(1 << 30) == 8 << 20


def test_numpy_and_c_sizing_agree():
    rng = random.Random(1)
    for L in [rng.randrange(1, 1 << 45) for _ in range(3000)] + list(range(1, 300)):
        assert co.piece_length(L) == zn.piece_length(L)
        assert co.get_k_and_m(L) == zn.get_k_and_m(L)


# ------------------------------------------- the reference's own tests
def _encode_chunk(chunk, idx):
    """encode_chunk semantics (piece.rs:320-361) on the oracle."""
    k, m = co.get_k_and_m(len(chunk))
    shares, B, pad = co.encode(k, m, chunk)
    return {"k": k, "m": m, "B": B, "padlen": pad, "chunk_idx": idx,
            "pieces": [(idx, i, shares[i]) for i in range(m)], "len": len(chunk)}


def test_reference_split_data_counts():
    # piece.rs:553-594: 1 MiB -> 4 chunks of 256 KiB, each k=2, m=3 -> 12.
    size = 1 << 20
    data = co.splitmix_bytes(5, size)
    cs = co.piece_length(size)
    assert cs == 256 << 10
    chunks = [_encode_chunk(data[i:i + cs], j) for j, i in enumerate(range(0, size, cs))]
    assert len(chunks) == 4
    expected = 0
    for c in chunks:
        ps = co.piece_length(c["len"])
        expected += c["m"] * -(-c["B"] // ps)
    assert sum(len(c["pieces"]) for c in chunks) == expected == 12


def test_reference_reconstruct_large_and_dropped():
    # piece.rs:597-649, with the erasure the reference test meant to apply
    # (its corrupted-case test drops nothing): keep 70 % of each chunk's
    # pieces in shuffled order and reconstruct.
    size = 1 << 20
    data = co.splitmix_bytes(6, size)
    cs = co.piece_length(size)
    rng = random.Random(3)
    out = []
    for j, i in enumerate(range(0, size, cs)):
        c = _encode_chunk(data[i:i + cs], j)
        keep = rng.sample(c["pieces"], int(np.ceil(len(c["pieces"]) * 0.7)))
        idx = [p[1] for p in keep]
        out.append(co.decode(c["k"], c["m"], [p[2] for p in keep], idx, c["B"], c["padlen"]))
    assert b"".join(out) == data.tobytes()


def test_reference_single_chunk_zeros():
    # piece.rs:652-689 on 1024 zero bytes; reduced set actually used here.
    d = np.zeros(1024, dtype=np.uint8)
    c = _encode_chunk(d, 0)
    assert (c["k"], c["m"]) == (1, 2)
    keep = c["pieces"][1:]  # only the parity piece survives
    assert co.decode(1, 2, [p[2] for p in keep], [1], c["B"], c["padlen"]) == d.tobytes()


def test_threaded_roundtrip_baseline_path():
    # bench.py's threaded CPU baseline leg: every chunk must round-trip.
    data = np.concatenate([co.splitmix_bytes(i, 12345) for i in range(12)])
    assert co.roundtrip_many(4, 6, data, 12345, 12, [0, 1], 4) == 0
    assert co.roundtrip_many(16, 24, data, 12345, 12, [0, 3, 5, 7, 9, 11, 13, 15], 3) == 0
    # losing more than n-k shares is a failure for every chunk
    assert co.roundtrip_many(4, 6, data, 12345, 12, [0, 1, 2], 2) == 12


def test_named_assumption_fixtures(golden):
    """Every behaviour pinned beyond fec.c (SURVEY 8(c) open item) is a named
    fixture a networked session can confirm against zfec-rs in one run; the
    oracle reproduces each, including the share order it is given."""
    names = {v["name"] for v in golden["assumptions"]}
    assert names == {"padlen_when_len_divisible_by_k", "padlen_when_len_not_divisible_by_k",
                     "decode_of_unsorted_shares", "n_equals_k", "k_1_replication"}
    for v in golden["assumptions"]:
        k, n = v["k"], v["n"]
        d = bytes.fromhex(v["data_hex"])
        shares, B, pad = co.encode(k, n, d)
        assert (B, pad) == (v["B"], v["padlen"]), v["name"]
        assert [bytes(s).hex() for s in shares[k:]] == v.get("parity_hex", []), v["name"]
        order = v["decode"].get("given_order", v["decode"].get("survivors"))
        rec = co.decode(k, n, [shares[i] for i in order], order, B, pad)
        assert sha(rec) == v["decode"]["data_sha256"] == sha(d), v["name"]


def test_decode_many_rebuilds_every_chunk():
    """The whole-batch oracle decode the BASELINE-size GPU tests check with
    (tests/batch_oracle.py): encode_parity_many then decode_many from data
    survivors and parity, for the config-3 erasure and a parity-only set."""
    import batch_oracle as BO
    for k, n, L, N, lost in ((8, 12, 4096, 6, (0, 3, 5)), (4, 6, 1024, 5, (9,)),
                             (16, 24, 2048, 3, tuple(range(8)))):
        B = L // k
        data = BO.splitmix_chunks(11, L, N)
        par = BO.parity_all(k, n, data, L, N)
        for i in range(N):
            want = co.encode(k, n, data[i * L:(i + 1) * L])[0][k:]
            assert np.array_equal(par[i * (n - k) * B:(i + 1) * (n - k) * B].reshape(n - k, B), want)
        surv = [i for i in range(n) if i not in lost][:k]
        wiped = data.copy().reshape(N, k, B)
        for e in lost:
            if e < k:
                wiped[:, e] = 0xA5
        out = BO.decode_all(k, n, wiped.reshape(-1), par, B, N, surv)
        assert BO.first_mismatch(out, data, L) is None
