"""C ABI library: loads, exports every declared symbol, host logic is right.

No GPU compute here: only the host-side entry points (parameter checks,
generator matrix, sizing) are called, plus the no-device error path.
"""
import ctypes
import os
import random
import re
import subprocess

import numpy as np
import pytest

from oracle import coracle as co
from storb_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "storb_rs.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(storb_\w+)\s*\(", src)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ["storb_rs_ctx_create", "storb_rs_encode", "storb_rs_decode",
              "storb_rs_encode_batch_dev", "storb_rs_decode_batch_dev", "storb_rs_apply_dev",
              "storb_piece_length", "storb_get_k_and_m", "storb_rs_strerror"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (storb_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_code():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_product_never_imports_the_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "storb_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
                text = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"(#|//).*", "", text).replace(
                    "oracle/", ""), f"{f} references the oracle"


def test_version_and_strerror():
    assert "gfx950" in _lib.version()
    L = _lib.lib()
    for code in range(6):
        assert L.storb_rs_strerror(code)


def test_check_params_matches_zfec_rules():
    for k, n, ok in [(1, 1, True), (1, 2, True), (4, 6, True), (256, 256, True), (0, 1, False),
            (0, 0, False), (3, 2, False), (2, 257, False), (1, 0, False)]:
        assert _lib.check_params(k, n) is ok, (k, n)


def test_product_generator_matches_oracle():
    # The product builds its generator independently (storb_amd/csrc/gf256.hpp).
    for k in range(1, 34):
        for n in range(k, min(k + 20, 257)):
            assert np.array_equal(_lib.enc_matrix(k, n), co.enc_matrix(k, n)), (k, n)
    for k, n in [(64, 96), (128, 192), (200, 256), (255, 256), (1, 256)]:
        assert np.array_equal(_lib.enc_matrix(k, n), co.enc_matrix(k, n)), (k, n)
    with pytest.raises(_lib.StorbRsError):
        _lib.enc_matrix(0, 3)


def test_block_size():
    for k, L in [(1, 13), (4, 1 << 20), (4, 10), (3, 1), (7, 100)]:
        assert _lib.block_size(k, L) == -(-L // k)


def test_sizing_matches_oracle():
    rng = random.Random(4)
    for L in [0, 1, 2, 9, 13, 16383, 16384, 16385] + [rng.randrange(1, 1 << 50) for _ in range(3000)]:
        assert _lib.piece_length(L) == co.piece_length(L), L
        if L:
            assert _lib.get_k_and_m(L) == co.get_k_and_m(L), L
    assert _lib.piece_length(1000, 4096, 8192) == co.piece_length(1000, 4096, 8192)


def test_no_device_is_an_error_not_a_fallback():
    if _lib.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.StorbRsError) as e:
        _lib.Context(-1)
    assert e.value.code == _lib.ENODEV


def test_device_numa_node_without_a_device():
    """storb_rs_device_numa_node: -1 for a device that is not there (it reads
    sysfs through the device's PCI bus id; nothing to read without one)."""
    if _lib.device_count() > 0:
        pytest.skip("a GPU is present")
    assert _lib.lib().storb_rs_device_numa_node(0) == -1
    assert _lib.lib().storb_rs_device_numa_node(7) == -1


def test_select_device_numa_topologies():
    """storb_rs_ctx_create(-1)'s device choice, on injected
    topologies with no device access: a thread's contexts go round-robin over
    the GPUs on its own socket, and over all GPUs when its socket has none or
    its node is unknown (upload.rs:418-420 through lib.rs:97-114)."""
    sel = _lib.select_device
    two_by_four = [0, 0, 0, 0, 1, 1, 1, 1]  # 2 sockets x 4 GPUs (an MI355X node)
    assert [sel(0, two_by_four, t) for t in range(9)] == [0, 1, 2, 3, 0, 1, 2, 3, 0]
    assert [sel(1, two_by_four, t) for t in range(5)] == [4, 5, 6, 7, 4]
    interleaved = [1, 0, 1, 0, 1, 0, 1, 0]
    assert [sel(0, interleaved, t) for t in range(4)] == [1, 3, 5, 7]
    assert [sel(1, interleaved, t) for t in range(4)] == [0, 2, 4, 6]
    # caller node unknown, or a node with no GPU: every GPU, plain round-robin
    assert [sel(-1, two_by_four, t) for t in range(9)] == list(range(8)) + [0]
    assert [sel(2, two_by_four, t) for t in range(8)] == list(range(8))
    # devices whose node is unknown (-1) are reachable only through the fallback
    assert [sel(0, [-1, 0, -1], t) for t in range(3)] == [1, 1, 1]
    assert [sel(-1, [-1, 0, -1], t) for t in range(3)] == [0, 1, 2]
    assert sel(0, [], 0) == -1
    # every GPU of the caller's socket gets an equal share of its contexts
    counts = [0] * 8
    for t in range(4000):
        counts[sel(1, two_by_four, t)] += 1
    assert counts == [0, 0, 0, 0, 1000, 1000, 1000, 1000]


def test_jit_compiles_decode_kernels_without_gpu():
    """The run-time-compiled decode kernels build with hipRTC on the host
    (no GPU): RS(16,8) with every data share lost, in place and assembled,
    RS(32,16) with 16 lost, k = 40 with 3 and with 18 lost (row-split).
    Matrices the policy does not want (RS(4,2),
    RS(8,4) with 3 lost, one lost share at k = 16) queue nothing."""
    from storb_amd import _lib
    before = _lib.jit_stats()
    _lib.jit_prepare_decode(4, 6, [2, 3, 4, 5])
    _lib.jit_prepare_decode(8, 12, [1, 2, 4, 6, 7, 8, 9, 10, 11])
    _lib.jit_prepare_decode(16, 24, list(range(1, 24)))  # 1 lost: table kernel
    assert _lib.jit_stats()["compiled"] == before["compiled"]
    _lib.jit_prepare_decode(16, 24, list(range(8, 24)))
    _lib.jit_prepare_decode(16, 24, [1, 2, 3, 5, 8, 13, 16, 17, 18, 19, 20, 21, 22, 23, 4, 6],
                            assemble=True)
    _lib.jit_prepare_decode(32, 48, list(range(16, 48)))
    # k > 32 (Storb's k = 64 for objects from ~160 GiB; a short last chunk
    # any k up to 64): one launch sees every input
    _lib.jit_prepare_decode(40, 60, [x for x in range(60) if x not in (1, 7, 30)])
    # 18 lost rows: one row-split kernel (two waves sharing planes through
    # LDS, rs_bitslice_core.h bs_split_body), with fused assembly
    _lib.jit_prepare_decode(40, 60, list(range(18, 60)), assemble=True)
    st = _lib.jit_stats()
    assert st["failed"] == 0 and st["pending"] == 0
    assert st["compiled"] == before["compiled"] + 5
    # the same pattern again is a cache hit
    _lib.jit_prepare_decode(16, 24, list(range(8, 24)))
    assert _lib.jit_stats()["compiled"] == st["compiled"]


def test_exit_with_jit_compiles_in_flight():
    """A process that exits while decode kernels are still queued or compiling
    exits cleanly: the JIT's exit hook (registered after hipRTC's own static
    state) fails the queued entries and waits out the compile in flight.
    Before, the compile ran on into comgr's destroyed state: an LLVM abort on
    the GPU box (tools/fuzz.py), a hang here."""
    import subprocess
    import sys
    code = (
        "import random\n"
        "from storb_amd import _lib\n"
        "rng = random.Random(7)\n"
        "for _ in range(6):\n"
        "    lost = rng.sample(range(32), rng.randint(2, 16))\n"
        "    _lib.jit_prepare_decode(32, 48, [x for x in range(48) if x not in lost])\n"
        "print('queued', _lib.jit_stats()['pending'])\n")
    env = dict(os.environ, PYTHONPATH=ROOT, AMD_COMGR_CACHE="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "queued" in r.stdout


def test_device_kernels_make_no_function_calls(tmp_path):
    """Every gfx950 kernel in the library is one inlined body: no s_swappc.
    An out-of-line call is how the 9-16-row descriptor kernel at k = 32 once
    compiled (uniform values in VGPRs, captures read through flat loads) --
    and it never finished on a 16-byte share (tools/fuzz.py seed 4242)."""
    import glob
    import shutil
    llvm = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(llvm):
        pytest.skip("llvm-objdump not installed")
    lib = tmp_path / "libstorb_rs.so"
    shutil.copy(_lib.LIB_PATH, lib)
    subprocess.run([llvm, "--offloading", str(lib)], cwd=tmp_path, check=True,
                   capture_output=True)
    objs = sorted(glob.glob(str(tmp_path / "*hipv4-amdgcn-amd-amdhsa--gfx950")))
    assert objs, "no gfx950 code objects in the library"
    for o in objs:
        dis = subprocess.run([llvm, "-d", "--mcpu=gfx950", o], capture_output=True, text=True,
                             check=True).stdout
        assert "s_swappc" not in dis, os.path.basename(o)
    # the library's own check agrees on every AOT code object
    for o in objs:
        r, why = _lib.code_object_calls(open(o, "rb").read())
        assert r == 0, (os.path.basename(o), why)


def _elf_symbols(b):
    """(file offset of the Elf64_Sym, name, type, size) of every .symtab entry."""
    import struct
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQII", b, shoff + i * shentsize) for i in range(shnum)]
    out = []
    for name, typ, _fl, _addr, off, size, link, _info in secs:
        if typ != 2:
            continue
        stroff = secs[link][4]
        for o in range(off + 24, off + size, 24):
            nm, info, _other, _shndx, _val, sz = struct.unpack_from("<IBBHQQ", b, o)
            end = b.index(b"\0", stroff + nm)
            out.append((o, b[stroff + nm:end].decode(), info & 0xF, sz))
    return out


def _jit_subprocess(code, tmp_path, **env):
    import sys
    e = dict(os.environ, PYTHONPATH=ROOT, STORB_RS_JIT_DUMP=str(tmp_path), **env)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def test_jit_refuses_kernels_that_call(tmp_path):
    """a run-time compiled kernel that makes a function call
    is refused before anything loads it (the round-4 hang was such a call,
    DESIGN.md §7). STORB_RS_JIT_TEST_CALL=1 gives every generated body an
    out-of-line callee: the compile thread refuses it, counts it, and the
    pattern keeps the table kernel (prepare reports the failure)."""
    import glob
    stats, err = _jit_subprocess(
        "import json\n"
        "from storb_amd import _lib\n"
        "try:\n"
        "    _lib.jit_prepare_decode(16, 24, list(range(8, 24)))\n"
        "except _lib.StorbRsError:\n"
        "    pass\n"
        "print(json.dumps(_lib.jit_stats()))\n", tmp_path, STORB_RS_JIT_TEST_CALL="1")
    assert stats["refused"] == 1 and stats["failed"] == 1 and stats["compiled"] == 0, stats
    assert "refused: out-of-line function" in err
    cos = glob.glob(str(tmp_path / "*.co"))
    assert len(cos) == 1
    b = bytearray(open(cos[0], "rb").read())
    r, why = _lib.code_object_calls(bytes(b))
    assert r == 1 and "storb_jit_test_callee" in why, why
    # Hide the callee's body from the symbol check (size 0): the disassembly
    # of the kernel still finds the call instruction itself.
    import struct
    callee = [s for s in _elf_symbols(b) if "storb_jit_test_callee" in s[1] and s[2] == 2]
    assert callee
    for off, _n, _t, _sz in callee:
        struct.pack_into("<Q", b, off + 16, 0)
    r, why = _lib.code_object_calls(bytes(b))
    assert r == 1 and "s_swappc" in why, why
    # not an ELF at all
    assert _lib.code_object_calls(b"\x00" * 128)[0] == -1


def test_jit_largest_kernels_make_no_calls(tmp_path):
    """The shipped JIT bodies at their largest: k = 64 with
    32 lost rows (one row-split launch) and with 2, k = 32 with 16 lost, k = 16
    with 8 lost assembled. All compile, none is refused, and every dumped code
    object passes the library's call check."""
    import glob
    stats, _ = _jit_subprocess(
        "import json\n"
        "from storb_amd import _lib\n"
        "_lib.jit_prepare_decode(64, 96, list(range(32, 96)))\n"
        "_lib.jit_prepare_decode(64, 96, list(range(2, 96)))\n"
        "_lib.jit_prepare_decode(32, 48, list(range(16, 48)))\n"
        "_lib.jit_prepare_decode(16, 24, list(range(8, 24)), assemble=True)\n"
        "print(json.dumps(_lib.jit_stats()))\n", tmp_path)
    assert stats["compiled"] == 4 and stats["refused"] == 0 and stats["failed"] == 0, stats
    cos = sorted(glob.glob(str(tmp_path / "*.co")))
    assert len(cos) == 4
    for c in cos:
        r, why = _lib.code_object_calls(open(c, "rb").read())
        assert r == 0, (c, why)


def test_marshal_chunks_arrays():
    """The arrays decode_chunks_raw hands storb_rs_decode_chunks: one address
    per share in chunk order, the share indices beside them, counts per chunk;
    non-uint8 / non-contiguous shares are converted (and kept alive)."""
    import numpy as np
    from storb_amd import _lib

    B = 64
    base = np.arange(3 * 4 * B, dtype=np.uint8).reshape(3, 4, B)
    odd = np.arange(2 * B, dtype=np.uint8)[::2]  # strided: copied
    chunks = [([base[0, 1], base[0, 3]], [1, 3]), ([base[1, 0], odd, bytes(B)], [0, 2, 5]),
              ([base[2, 2]], [4])]
    ptrs, idx, cnt, keep = _lib.marshal_chunks(chunks, B)
    assert ptrs.dtype == np.uint64 and idx.dtype == np.uint32 and cnt.dtype == np.uint32
    assert cnt.tolist() == [2, 3, 1] and idx.tolist() == [1, 3, 0, 2, 5, 4]
    assert ptrs[0] == base[0, 1].ctypes.data and ptrs[1] == base[0, 3].ctypes.data
    assert ptrs[2] == base[1, 0].ctypes.data and ptrs[5] == base[2, 2].ctypes.data
    assert len(keep) == 6 and keep[3].flags.c_contiguous and keep[3].ctypes.data == ptrs[3]
    assert bytes(keep[3]) == bytes(odd) and keep[4].ctypes.data == ptrs[4]
