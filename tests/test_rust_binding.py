"""The zfec-rs shim (integration/zfec-rs-mi355x/src/lib.rs) pinned to the C ABI.

No Rust toolchain exists in this image, so the one binding the tier is about
(Storb -> zfec-rs API -> storb_rs.h, piece.rs:9,328-329,375,383-386) is held
in place mechanically (VERDICT r2 'next' 4):

* every `extern "C"` declaration in lib.rs is parsed and checked against the
  prototype of the same name in include/storb_rs.h -- name, arity, and every
  parameter and return type mapped (u32 <-> uint32_t, usize <-> size_t,
  c_int <-> int, pointer constness level by level);
* the shim's Fec::new / encode / decode are transliterated (tests/shim_mirror.py)
  and run on the assumption fixtures: on CPU against the oracle behind the C
  ABI's contract, on the GPU against libstorb_rs.so itself.
"""
import json
import os
import re

import numpy as np
import pytest

import shim_mirror as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRATE_SRC = os.path.join(ROOT, "integration", "zfec-rs-mi355x", "src")
LIB_RS = os.path.join(CRATE_SRC, "lib.rs")
MI355X_RS = os.path.join(CRATE_SRC, "mi355x.rs")
HEADER = os.path.join(ROOT, "include", "storb_rs.h")
GOLDEN = os.path.join(ROOT, "tests", "golden", "zfec_vectors.json")

C_BASE = {"int": "c_int", "uint32_t": "u32", "size_t": "usize", "uint8_t": "u8",
          "char": "c_char", "uint64_t": "u64", "void": "c_void",
          "storb_rs_ctx": "StorbRsCtx", "storb_rs_op": "StorbRsOp",
          "storb_rs_jit_stats_t": "StorbRsJitStats", "storb_rs_ctx_stats_t": "StorbRsCtxStats",
          "storb_rs_notify_fn": 'Option<unsafe extern "C" fn(*mut c_void)>'}


def c_type_to_rust(ctype: str) -> str:
    """A C parameter type as the Rust FFI type it must be declared with.
    `T *const *` is a pointer to a const pointer: `*const *mut T`."""
    toks = re.findall(r"\*|const|\w+", ctype)
    base_const = False
    base = None
    i = 0
    while i < len(toks) and toks[i] != "*":
        if toks[i] == "const":
            base_const = True
        else:
            base = toks[i]
        i += 1
    assert base in C_BASE, f"unmapped C type {ctype!r}"
    t, cur_const = C_BASE[base], base_const
    for tok in toks[i:]:
        if tok == "*":
            t = ("*const " if cur_const else "*mut ") + t
            cur_const = False
        else:  # const qualifying the pointer just built (its pointee, for the next *)
            cur_const = True
    return t


def header_prototypes() -> dict:
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(storb_\w+)\s*\(([^;{]*?)\)\s*;", src):
        ret, name, params = m.group(1).strip(), m.group(2), m.group(3).strip()
        plist = []
        if params and params != "void":
            for p in params.split(","):
                p = p.strip()
                arr = re.match(r"(.*?)(\w+)\s*\[\s*\d*\s*\]$", p)
                if arr:  # `uint8_t out[32]` decays to a pointer
                    plist.append(c_type_to_rust(arr.group(1) + " *"))
                    continue
                pm = re.match(r"(.*?[\s\*])(\w+)$", p)
                plist.append(c_type_to_rust(pm.group(1) if pm else p))
        protos[name] = (None if ret == "void" else c_type_to_rust(ret), plist)
    return protos


def rust_externs(path=LIB_RS) -> dict:
    """Every storb_* function of every `extern "C"` block of one source file
    (the glibc eventfd/close block of mi355x.rs is not the ABI's)."""
    src = open(path).read()
    out = {}
    for block in re.findall(r'extern "C" \{(.*?)\n\}', src, re.S):
        for m in re.finditer(r"fn\s+(\w+)\s*\((.*?)\)\s*(->\s*([^;]+))?;", block, re.S):
            name, params, ret = m.group(1), m.group(2), m.group(4)
            if not name.startswith("storb_"):
                continue
            plist = []
            for p in [x.strip() for x in params.split(",") if x.strip()]:
                _, ty = p.split(":", 1)
                plist.append(" ".join(ty.split()))
            out[name] = (ret.strip() if ret else None, plist)
    return out


def test_c_type_mapping_rules():
    assert c_type_to_rust("uint8_t *const *") == "*const *mut u8"
    assert c_type_to_rust("const uint8_t *const *") == "*const *const u8"
    assert c_type_to_rust("const uint32_t *") == "*const u32"
    assert c_type_to_rust("storb_rs_ctx **") == "*mut *mut StorbRsCtx"
    assert c_type_to_rust("const storb_rs_ctx *") == "*const StorbRsCtx"
    assert c_type_to_rust("size_t *") == "*mut usize"
    assert c_type_to_rust("const char *") == "*const c_char"


def _check_against_header(rs):
    hdr = header_prototypes()
    for name, (ret, params) in rs.items():
        assert name in hdr, f"{name} is not declared in include/storb_rs.h"
        hret, hparams = hdr[name]
        assert len(params) == len(hparams), (name, params, hparams)
        for i, (r, h) in enumerate(zip(params, hparams)):
            assert r == h, f"{name} parameter {i}: Rust {r!r} vs header {h!r}"
        assert ret == hret, f"{name} return: Rust {ret!r} vs header {hret!r}"


def test_every_rust_extern_matches_the_header():
    rs = rust_externs(LIB_RS)
    # the zfec-rs API (Fec::new / encode / decode) binds exactly these eight
    assert set(rs) == {"storb_rs_ctx_create", "storb_rs_ctx_destroy", "storb_rs_strerror",
                       "storb_rs_last_error", "storb_rs_check_params", "storb_rs_block_size",
                       "storb_rs_encode_shares", "storb_rs_decode"}, sorted(rs)
    _check_against_header(rs)


def test_mi355x_module_externs_match_the_header():
    """the batch, hashed, async and page-locked calls an
    integrator wires into upload.rs:418-420 / download.rs:464 have a pinned
    Rust surface (zfec_rs::mi355x)."""
    rs = rust_externs(MI355X_RS)
    want = {"storb_rs_encode_chunks", "storb_rs_encode_chunks_hashed", "storb_rs_decode_chunks",
            "storb_rs_encode_async", "storb_rs_decode_async", "storb_rs_op_test",
            "storb_rs_op_finish", "storb_rs_notify_fd", "storb_rs_host_alloc",
            "storb_rs_host_free", "storb_rs_host_register", "storb_rs_host_unregister",
            "storb_blake3"}
    assert want <= set(rs), sorted(want - set(rs))
    _check_against_header(rs)
    assert "pub mod mi355x;" in open(LIB_RS).read()


def test_header_parser_sees_the_whole_abi():
    hdr = header_prototypes()
    # spot checks that the parser is not silently skipping prototypes
    assert hdr["storb_rs_decode"][1] == ["*mut StorbRsCtx", "u32", "u32", "*const *const u8",
                                         "*const u32", "u32", "usize", "usize", "*mut u8"]
    assert hdr["storb_rs_ctx_destroy"] == (None, ["*mut StorbRsCtx"])
    assert hdr["storb_blake3"][1] == ["*const u8", "usize", "*mut u8"]
    names = set(re.findall(r"\b(storb_[a-z0-9_]+)\(", open(HEADER).read()))
    assert set(hdr) == names, names ^ set(hdr)


def _assumptions():
    return json.load(open(GOLDEN))["assumptions"]


def _run_fixtures(backend):
    for fx in _assumptions():
        k, n = fx["k"], fx["n"]
        data = bytes.fromhex(fx["data_hex"])
        fec = S.Fec(k, n, backend)
        chunks, pad = fec.encode(data)
        B = fx["B"]
        assert pad == fx["padlen"], fx["name"]
        assert [c.index for c in chunks] == list(range(n))
        assert all(len(c.data) == B for c in chunks)
        padded = data + bytes(k * B - len(data))
        for j in range(k):
            assert bytes(chunks[j].data) == padded[j * B:(j + 1) * B], (fx["name"], j)
        assert [bytes(c.data).hex() for c in chunks[k:]] == fx["parity_hex"], fx["name"]
        dec = fx["decode"]
        order = dec.get("given_order") or dec["survivors"]
        pieces = [(i, bytes(chunks[i].data)) for i in order]
        got = S.decode_chunk(pieces, k, n, pad, backend)
        assert got == data, fx["name"]


def test_shim_on_assumption_fixtures_cpu():
    _run_fixtures(S.OracleBackend())


def test_shim_checks_cpu():
    be = S.OracleBackend()
    for k, m in ((0, 2), (3, 2), (257, 300), (4, 257)):
        with pytest.raises(S.ShimError) as e:
            S.Fec(k, m, be)
        assert e.value.code == S.EINVAL
    fec = S.Fec(4, 6, be)
    chunks, pad = fec.encode(b"0123456789abcdef!")  # 17 bytes: B = 5, pad 3
    assert pad == 3
    with pytest.raises(S.ShimError) as e:  # fewer than k shares
        fec.decode(chunks[:3], pad)
    assert e.value.code == S.ENOTENOUGH
    with pytest.raises(S.ShimError) as e:  # padding >= k*b
        fec.decode(chunks[:4], 20)
    assert e.value.code == S.EINVAL
    bad = [S.Chunk(bytearray(c.data), c.index) for c in chunks[:4]]
    bad[2].data = bad[2].data[:4]
    with pytest.raises(S.ShimError) as e:  # shares of unequal length
        fec.decode(bad, pad)
    assert e.value.code == S.EINVAL
    with pytest.raises(S.ShimError) as e:  # b == 0
        fec.decode([S.Chunk(bytearray(), i) for i in range(4)], 0)
    assert e.value.code == S.EINVAL
    with pytest.raises(S.ShimError) as e:  # empty chunk: storb_rs_encode_shares EINVAL
        fec.encode(b"")
    assert e.value.code == S.EINVAL


def test_shim_random_roundtrips_through_parity_cpu():
    be = S.OracleBackend()
    rng = np.random.default_rng(3)
    for k, n in ((2, 3), (4, 6), (8, 12), (5, 9)):
        for ln in (1, 7, 1000, 4097):
            data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            fec = S.Fec(k, n, be)
            chunks, pad = fec.encode(data)
            surv = sorted(rng.choice(n, size=k, replace=False).tolist())
            got = S.decode_chunk([(i, bytes(chunks[i].data)) for i in surv[::-1]], k, n, pad, be)
            assert got == data, (k, n, ln, surv)


@pytest.mark.gpu
def test_shim_on_assumption_fixtures_gpu(ctx):
    _run_fixtures(S.LibBackend(ctx.handle))


@pytest.mark.gpu
def test_shim_random_roundtrips_gpu_vs_oracle(ctx):
    lib_be, ora = S.LibBackend(ctx.handle), S.OracleBackend()
    rng = np.random.default_rng(4)
    for k, n in ((2, 3), (4, 6), (8, 12), (16, 24), (6, 9)):
        for ln in (13, 4096 * k + 5, 1 << 18):
            data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            got, gpad = S.Fec(k, n, lib_be).encode(data)
            want, wpad = S.Fec(k, n, ora).encode(data)
            assert gpad == wpad and [bytes(c.data) for c in got] == [bytes(c.data) for c in want]
            surv = sorted(rng.choice(n, size=min(n, k + 1), replace=False).tolist())
            pieces = [(i, bytes(got[i].data)) for i in surv[::-1]]
            assert S.decode_chunk(pieces, k, n, gpad, lib_be) == data, (k, n, ln, surv)
