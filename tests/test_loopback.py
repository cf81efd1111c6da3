"""Config 5 harness and Storb's wire formats (storb_amd/wire.py).

CPU: a real miner process (tools/loopback.py miner) stores pieces sent with
the store framing (upload.rs:88-100), acks blake3, serves them back as a
bincode PieceResponse (routes.rs:188-206) that the validator side parses and
verifies (download.rs:121-164); the on-disk layout is <hash[0:2]>/<hash[2:]>.
GPU: the full loop at reduced size, bit-exact, with a killed miner.
"""
import argparse
import http.client
import os
import socket
import struct
import subprocess
import sys

import pytest

from oracle.blake3_ref import blake3 as ref
from storb_amd import wire

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_piece_response_format():
    h = ref(b"xyz")
    body = wire.serialise_piece_response(h, b"xyz")
    assert body == h + struct.pack("<Q", 3) + b"xyz"
    assert wire.deserialise_piece_response(body, h) == b"xyz"
    with pytest.raises(ValueError):
        wire.deserialise_piece_response(body + b"!", h)  # reject_trailing_bytes
    with pytest.raises(ValueError):
        wire.deserialise_piece_response(wire.serialise_piece_response(h, b"xyw"), h)


def test_object_store_mirrors_reference_tests(tmp_path):
    """crates/storb_miner/src/store.rs:70-182: creating a store (fresh and
    existing directory), writing a piece to <hash[0:2]>/<hash[2:]> (the
    folder is created if an existing store lacks it), reading it back,
    overwriting it."""
    p = str(tmp_path / "store")
    s = wire.ObjectStore(p)
    assert os.path.isdir(p)
    s2 = wire.ObjectStore(p)  # existing directory
    assert os.path.isdir(s2.path)
    bare = tmp_path / "bare"
    bare.mkdir()
    wire.ObjectStore(str(bare)).write("ab" + "0" * 62, b"x")  # no hex folders yet
    assert (bare / "ab" / ("0" * 62)).read_bytes() == b"x"
    data = os.urandom(1000)
    hx = ref(data).hex()
    f = s.write(hx, data)
    assert f == os.path.join(p, hx[:2], hx[2:]) and os.path.exists(f)
    assert s.read(hx) == data
    data2 = os.urandom(1000)
    s.write(hx, data2)
    assert s.read(hx) == data2 and s.read(hx) != data


def test_miner_store_and_retrieve(tmp_path):
    sp, hp = free_port(), free_port()
    store = tmp_path / "m0"
    proc = subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "loopback.py"), "miner",
                             "--store-port", str(sp), "--http-port", str(hp), "--dir", str(store)],
                            stdout=subprocess.PIPE, text=True)
    try:
        assert proc.stdout.readline().strip() == "ready"
        s = socket.create_connection(("127.0.0.1", sp))
        pieces = [os.urandom(n) for n in (1, 1000, 70000, 262144)]
        acks = [wire.send_piece(s, bytes(96), p) for p in pieces]
        s.close()
        assert acks == [ref(p) for p in pieces]
        for p, h in zip(pieces, acks):
            hx = h.hex()
            assert (store / hx[:2] / hx[2:]).read_bytes() == p
            c = http.client.HTTPConnection("127.0.0.1", hp, timeout=10)
            c.request("GET", f"/piece?piecehash={hx}&handshake={bytes(96).hex()}")
            r = c.getresponse()
            assert r.status == 200
            assert wire.deserialise_piece_response(r.read(), h) == p
            c.close()
        c = http.client.HTTPConnection("127.0.0.1", hp, timeout=10)
        c.request("GET", f"/piece?piecehash={'00' * 32}&handshake=00")
        assert c.getresponse().status == 500
        # the harness's keep-alive client: every piece over one connection,
        # then a missing one, then a good one again on the same connection
        pc = wire.PieceClient("127.0.0.1", hp)
        for p, h in list(zip(pieces, acks)) * 2:
            st, body = pc.get(h.hex(), bytes(96).hex())
            assert st == 200 and wire.deserialise_piece_response(body, h) == p
        assert pc.get("00" * 32, "00")[0] == 500
        st, body = pc.get(acks[0].hex(), "00")
        assert st == 200 and wire.deserialise_piece_response(body, acks[0]) == pieces[0]
        pc.close()
    finally:
        proc.kill()
        proc.wait()


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [0, 3])
def test_loopback_roundtrip_small(gpus):
    """gpus=3: the chunks partition over three contexts (several per device
    on a one-GPU box), the config-5 layout for 8 x MI355X."""
    import loopback
    res = loopback.run(argparse.Namespace(size=(24 << 20) + 12345, miners=4, seed=1,
                                          kill_seed=7, gpus=gpus, cold=False))
    assert res["bit_exact"]
    assert res["ack_mismatch"] == 0
    assert res["chunks_decoded_through_parity"] > 0
    assert res["contexts"] == (gpus or max(1, res["visible_gpus"]))


@pytest.mark.gpu
def test_loopback_config5_geometry():
    """BASELINE config 5 at its own geometry: a 640 MiB (+ tail) object cut by
    Storb's own rule (upload.rs:209 piece_length) into 8 MiB chunks, each
    k=16, m=24 (piece.rs:307-317), over 8 miners with one killed. Every piece
    a miner stored and every piece id (computed on the GPU, and acked by the
    miners over the store framing) is checked against the oracle's shares;
    the host hasher used for that is pinned to the reference blake3
    (test_blake3.py), which is also run itself on a sample of pieces."""
    import loopback
    from oracle import coracle
    from storb_amd import _lib
    size = (640 << 20) + 12345
    seen = {}

    def inspect(obj, metas, dirs):
        geo = [(m["k"], m["m"], m["B"]) for m in metas]
        assert geo.count((16, 24, 512 << 10)) == 80 and len(geo) == 81
        for ci, meta in enumerate(metas):
            chunk = obj[meta["off"]:meta["off"] + meta["len"]]
            shares, B, pad = coracle.encode(meta["k"], meta["m"], chunk)
            assert (B, pad) == (meta["B"], meta["padlen"])
            for i in range(meta["m"]):
                h = meta["hashes"][i]
                assert h == _lib.blake3(shares[i]), (ci, i)
                hx = h.hex()
                with open(os.path.join(dirs[meta["miner"][i]], hx[:2], hx[2:]), "rb") as f:
                    assert f.read() == shares[i].tobytes(), (ci, i)
                if (ci, i) in ((0, 0), (0, 23), (40, 17)):
                    assert ref(shares[i].tobytes()) == h, (ci, i)
                    seen[(ci, i)] = True

    res = loopback.run(argparse.Namespace(size=size, miners=8, seed=3, kill_seed=7, gpus=0,
                                          cold=False), inspect=inspect)
    assert len(seen) == 3
    assert res["bit_exact"] and res["ack_mismatch"] == 0
    assert [16, 24] in [list(x) for x in res["k_m"]] or (16, 24) in res["k_m"]
    assert res["chunk_bytes"] == 8 << 20
    assert res["chunks_decoded_through_parity"] > 0
