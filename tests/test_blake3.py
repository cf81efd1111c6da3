"""BLAKE3 shard identity (Storb: upload.rs:623, miner lib.rs:265-283,
download.rs:158-161; crate blake3 1.8.2).

Pins: the published BLAKE3 vectors -- hash of the empty input and of "abc",
and entries of the official test_vectors.json (input byte i = i % 251) --
against the restated reference (oracle/blake3_ref.py); then the product's host
hasher and its gfx950 batch kernel against that reference, bit-exact.
"""
import os
import random

import numpy as np
import pytest

from oracle.blake3_ref import blake3 as ref
from storb_amd import _lib


def tv(n):
    return bytes(i % 251 for i in range(n))


PUBLISHED = {
    # official test_vectors.json, 32-byte hash mode outputs
    0: "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
    1: "2d3adedff11b61f14c886e35afa036736dcd87a74d27b5c1510225d0f592e213",
    1023: "10108970eeda3eb932baac1428c7a2163b0e924c9a9e25b35bba72b28f70bd11",
    1024: "42214739f095a406f3fc83deb889744ac00df831c10daa55189b5d121c855af7",
    1025: "d00278ae47eb27b34faecf67b4fe263f82d5412916c1ffd97c8cb7fb814b8444",
}


def test_reference_matches_published_vectors():
    assert ref(b"abc").hex() == "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"
    for n, h in PUBLISHED.items():
        assert ref(tv(n)).hex() == h, n


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 2049, 3072,
                               3073, 4096, 4097, 5121, 8193, 16384, 31744, 102400])
def test_host_hasher_matches_reference(n):
    assert _lib.blake3(tv(n)) == ref(tv(n))


@pytest.mark.parametrize("n", [16 * 1024 + 1, 17 * 1024, 33 * 1024, 33 * 1024 + 1, 65 * 1024,
                               (256 << 10) + 1, (512 << 10) + 1024, (1 << 20) + 1])
def test_host_hasher_simd_subtrees(n):
    """Sizes whose first n-1 chunks decompose into subtrees of >= 16 chunks:
    the AVX-512 path (16 chunks and 16 parents per compression) where the
    CPU has it, against the restated reference."""
    d = random.Random(n).randbytes(n)
    assert _lib.blake3(d) == ref(d)


def test_host_hasher_simd_equals_scalar_large():
    """Up to 9 MiB (Storb's 8 MiB shard sizing and beyond): the SIMD hasher
    against the scalar compression of the same library (STORB_B3_SCALAR=1 in
    a child process), which the tests above pin to the reference."""
    import subprocess
    import sys
    sizes = [(8 << 20), (8 << 20) + 3, (9 << 20) - 1024 * 17 + 5, (2 << 20) + 1024 * 31]
    rng = np.random.default_rng(11)
    data = [rng.bytes(n) for n in sizes]
    mine = [_lib.blake3(d).hex() for d in data]
    code = ("import sys, numpy as np; from storb_amd import _lib; "
            "rng = np.random.default_rng(11); "
            f"print(' '.join(_lib.blake3(rng.bytes(n)).hex() for n in {sizes}))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, STORB_B3_SCALAR="1")
    out = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, check=True,
                         capture_output=True, text=True).stdout.split()
    assert out == mine


def test_host_hasher_random_sizes():
    rng = random.Random(3)
    for _ in range(12):
        n = rng.randrange(0, 200000)
        d = rng.randbytes(n)
        assert _lib.blake3(d) == ref(d)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("length,count,stride,offset", [
    (0, 3, 16, 0), (1, 5, 16, 0), (64, 4, 64, 0), (1000, 3, 1024, 0), (1024, 4, 1024, 0),
    (1025, 3, 1040, 0), (4099, 3, 4112, 3), (256 << 10, 6, 256 << 10, 0),
    (300 * 1024 + 5, 2, 300 * 1024 + 16, 0), (1 << 20, 3, 1 << 20, 0),
    ((1 << 20) + 17, 2, (1 << 20) + 32, 1), (4 << 20, 2, 4 << 20, 0), (16 << 20, 1, 16 << 20, 0),
    # several shards per workgroup (segments of 1..32 lanes), counts that
    # leave the last workgroup partly empty
    (100, 1000, 112, 0), (2048, 300, 2048, 0), (3 * 1024 + 1, 257, 4096, 0),
    (16 << 10, 77, 16 << 10, 0), (64 << 10, 33, 64 << 10, 0), (5 * 1024, 9, 5 * 1024 + 16, 3),
    (127 * 1024, 5, 127 * 1024, 0)])
def test_device_batch_matches_host(ctx, length, count, stride, offset):
    import torch
    host = np.frombuffer(np.random.default_rng(length + count).bytes(count * stride + offset + 16),
                         dtype=np.uint8).copy()
    d = torch.from_numpy(host).to("cuda:0")
    out = torch.zeros(count * 32, dtype=torch.uint8, device="cuda:0")
    ctx.blake3_batch_dev(d.data_ptr() + offset, length, count, stride, out.data_ptr())
    got = out.cpu().numpy().reshape(count, 32)
    for i in range(count):
        msg = host[offset + i * stride: offset + i * stride + length].tobytes()
        assert got[i].tobytes() == _lib.blake3(msg), (length, i)
    if length <= 1 << 20:
        assert got[0].tobytes() == ref(host[offset:offset + length].tobytes())


@pytest.mark.gpu
def test_device_hashes_of_encoded_shards(ctx):
    """Storb's piece hashes for a batch of RS(4,2) 1 MiB chunks, computed where
    encode left the shards, equal blake3 of the host-side shards."""
    import torch
    from oracle import coracle
    k, n, L, N = 4, 6, 1 << 20, 8
    B = L // k
    data = torch.empty(N * L, dtype=torch.uint8, device="cuda:0")
    par = torch.empty(N * (n - k) * B, dtype=torch.uint8, device="cuda:0")
    ctx.fill_splitmix_dev(data.data_ptr(), L, N, L, 0x5709B)
    ctx.encode_batch_dev(k, n, B, N, data.data_ptr(), par.data_ptr())
    hd = torch.empty(N * k * 32, dtype=torch.uint8, device="cuda:0")
    hp = torch.empty(N * (n - k) * 32, dtype=torch.uint8, device="cuda:0")
    ctx.blake3_batch_dev(data.data_ptr(), B, N * k, B, hd.data_ptr())
    ctx.blake3_batch_dev(par.data_ptr(), B, N * (n - k), B, hp.data_ptr())
    hd = hd.cpu().numpy().reshape(N, k, 32)
    hp = hp.cpu().numpy().reshape(N, n - k, 32)
    for s in (0, N - 1):
        shares, _, _ = coracle.encode(k, n, coracle.splitmix_bytes(0x5709B + s, L))
        for i in range(n):
            want = _lib.blake3(shares[i].tobytes())
            got = hd[s, i] if i < k else hp[s, i - k]
            assert got.tobytes() == want, (s, i)


def _hashed_case(ctx, k, n, B, N, seed, data_stride=0, parity_stride=0, check_all=True):
    """storb_rs_encode_hashed_dev on N stripes of splitmix data: parity against
    the oracle's encode, every digest against the host blake3 of that share."""
    import torch
    from oracle import coracle
    ds = data_stride or k * B
    ps = parity_stride or (n - k) * B
    data = torch.zeros(N * ds, dtype=torch.uint8, device="cuda:0")
    par = torch.full((N * ps,), 0xA5, dtype=torch.uint8, device="cuda:0")
    hashes = torch.full((N * n * 32,), 0x5A, dtype=torch.uint8, device="cuda:0")
    ctx.fill_splitmix_dev(data.data_ptr(), k * B, N, ds, seed)
    ctx.encode_hashed_dev(k, n, B, N, data.data_ptr(), par.data_ptr(), hashes.data_ptr(),
                          data_stride, parity_stride)
    torch.cuda.synchronize()
    par = par.cpu().numpy()
    got = hashes.cpu().numpy().reshape(N, n, 32)
    stripes = range(N) if check_all else sorted({0, 1, N // 2, N - 1})
    for s in stripes:
        shares, _, _ = coracle.encode(k, n, coracle.splitmix_bytes(seed + s, k * B))
        for i in range(k, n):
            o = s * ps + (i - k) * B
            assert np.array_equal(par[o:o + B], shares[i]), (k, n, B, s, i)
        for t in range(n):
            assert got[s, t].tobytes() == _lib.blake3(shares[t].tobytes()), (k, n, B, s, t)
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("k,n,B,N", [
    (4, 6, 256 << 10, 6),   # Storb's 1 MiB chunk: 256 chunks per share, one stripe per workgroup
    (4, 6, 128 << 10, 5),   # 512 KiB chunks (config 1): two stripes per workgroup, one dead
    (2, 3, 128 << 10, 7),   # the storb-faithful 256 KiB chunk of config 4
    (4, 6, 1 << 10, 300),   # one chunk per share: the chunk is the root
    (4, 6, 3 << 10, 100),   # 3 chunks: the odd node carried up
    (2, 3, 5 << 10, 77),    # 5 chunks, 51 stripes per workgroup
    (4, 6, 255 << 10, 3),   # 255 chunks
    (4, 6, 2 << 10, 1)])
def test_encode_hashed_dev_fused_kernel(ctx, k, n, B, N):
    _hashed_case(ctx, k, n, B, N, 0x5709B + B + N, check_all=N * B <= (8 << 20))


@pytest.mark.gpu
def test_encode_hashed_dev_strided_and_unfused_geometries(ctx):
    # pitched stripes (fused kernel); geometries without a fused kernel run
    # encode then hash and scatter the digests into the same layout
    _hashed_case(ctx, 4, 6, 64 << 10, 9, 11, data_stride=(4 << 16) + 4096,
                 parity_stride=(2 << 16) + 512)
    _hashed_case(ctx, 16, 24, 32 << 10, 5, 12)
    _hashed_case(ctx, 4, 6, 1000, 4, 13)          # not a multiple of 1 KiB
    _hashed_case(ctx, 4, 6, 512 << 10, 2, 14)     # over 256 KiB per share
    _hashed_case(ctx, 3, 5, 4 << 10, 3, 15)


@pytest.mark.gpu
def test_encode_hashed_dev_fused_equals_two_kernel_path(monkeypatch):
    """STORB_RS_FUSED_HASH=0 (encode kernel, then hash kernel) and the fused
    kernel give the same parity and digests, and the batch entry point
    (storb_rs_encode_chunks_hashed) returns them too."""
    import torch
    k, n, B, N = 4, 6, 256 << 10, 12
    outs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("STORB_RS_FUSED_HASH", fused)
        c = _lib.Context(0)
        try:
            data = torch.empty(N * k * B, dtype=torch.uint8, device="cuda:0")
            par = torch.empty(N * (n - k) * B, dtype=torch.uint8, device="cuda:0")
            h = torch.empty(N * n * 32, dtype=torch.uint8, device="cuda:0")
            c.fill_splitmix_dev(data.data_ptr(), k * B, N, k * B, 99)
            c.encode_hashed_dev(k, n, B, N, data.data_ptr(), par.data_ptr(), h.data_ptr())
            torch.cuda.synchronize()
            host = data.cpu().numpy()
            p2, h2 = c.encode_chunks_hashed(k, n, host, k * B, N)
            outs.append((par.cpu().numpy(), h.cpu().numpy(), np.asarray(p2).ravel(),
                         np.asarray(h2).ravel()))
        finally:
            c.close()
    (pa, ha, pb, hb), (qa, ga, qb, gb) = outs
    assert np.array_equal(pa, qa) and np.array_equal(ha, ga)
    assert np.array_equal(pa, pb) and np.array_equal(ha, hb)
    assert np.array_equal(qa, qb) and np.array_equal(ga, gb)


@pytest.mark.gpu
def test_device_batch_rejects_oversize(ctx):
    with pytest.raises(_lib.StorbRsError) as e:
        ctx.blake3_batch_dev(0, (16 << 20) + 1, 1, 0, 0)
    assert e.value.code == _lib.EINVAL


@pytest.mark.gpu
@pytest.mark.parametrize("pinned_out", [True, False])
def test_encode_chunks_hashed_zero_copy(ctx, pinned_out):
    """storb_rs_encode_chunks_hashed from page-locked chunks (DMA'd in place,
    parity written in place when the output is page-locked too, else through
    staging), the fused kernel on the device: oracle parity, host blake3 of
    every share."""
    from oracle import coracle
    k, n, L, N = 4, 6, 1 << 20, 5
    B = L // k
    src = _lib.PinnedBuffer(N * L)
    src.array[:] = np.frombuffer(np.random.default_rng(77).bytes(N * L), dtype=np.uint8)
    if pinned_out:
        dst = _lib.PinnedBuffer(N * (n - k) * B)
        out = dst.array
    else:
        out = np.empty(N * (n - k) * B, np.uint8)
    out[:] = 0
    ids = np.zeros((N, n, 32), np.uint8)
    par, ids = ctx.encode_chunks_hashed(k, n, src.array, L, N, out=out, hashes=ids)
    for c in range(N):
        shares, _, _ = coracle.encode(k, n, src.array[c * L:(c + 1) * L])
        for i in range(k, n):
            o = (c * (n - k) + i - k) * B
            assert np.array_equal(par[o:o + B], shares[i]), (c, i)
        for t in range(n):
            assert ids[c, t].tobytes() == _lib.blake3(shares[t].tobytes()), (c, t)


@pytest.mark.gpu
@pytest.mark.parametrize("k,n,L,cnt", [
    (4, 6, 4 * 1001 + 3, 9),       # B = 1002: shares pitched 1008 apart in staging, last padded
    (16, 24, 16 * 4099 + 5, 5),    # no fused kernel: one hash launch over every share
    (2, 3, 2 * 333, 4),            # B < one 1 KiB chunk
])
def test_encode_chunks_hashed_pitched_staging(ctx, k, n, L, cnt):
    """storb_rs_encode_chunks_hashed where the share size is not a multiple of
    16 bytes: the staged shares sit S = round_up(B, 16) apart, so the hash
    launch covers len = B at pitch S (launch_blake3_stripes), and every
    digest -- data and parity, in [chunk][share] order -- is the host blake3
    of the oracle's (zero-padded) share."""
    from oracle import coracle
    B = -(-L // k)
    host = np.concatenate([coracle.splitmix_bytes(0x5709B + 77 * c, L) for c in range(cnt)])
    par, ids = ctx.encode_chunks_hashed(k, n, host, L, cnt)
    par = np.asarray(par).reshape(cnt, n - k, B)
    ids = np.asarray(ids).reshape(cnt, n, 32)
    for c in range(cnt):
        shares, _, _ = coracle.encode(k, n, host[c * L:(c + 1) * L])
        assert np.array_equal(par[c], np.asarray(shares[k:]).reshape(n - k, B)), (k, n, c)
        for t in range(n):
            assert ids[c, t].tobytes() == _lib.blake3(np.asarray(shares[t]).tobytes()), (c, t)
