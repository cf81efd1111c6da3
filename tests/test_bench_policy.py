"""bench.py's mirror of the JIT launch policy (which kernel name and how many
launches a leg has) must follow rs_args.h bs_split / rs_jit.cpp row blocks,
or the bench line's kernel names, launch counts and PMC matches go wrong."""
import importlib.util
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("storb_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bs_split_rule_is_the_one_mirrored():
    src = open(os.path.join(ROOT, "storb_amd", "csrc", "rs_args.h")).read()
    m = re.search(r"constexpr bool bs_split\(int K, int R\) \{ return ([^;]+); \}", src)
    assert m, "bs_split not found in rs_args.h"
    assert m.group(1) == "K % kSplitGroup == 0 && R > 16 && R <= 32"
    assert re.search(r"constexpr int kSplitGroup = 2;", src)


def test_jit_blocks_match_row_split_and_row_blocks():
    bench = load_bench()
    for k in (8, 12, 16, 17, 24, 40, 41, 63, 64):
        for rows in range(1, 33):
            if k % 2 == 0 and 16 < rows <= 32:
                want = (1, rows)
            else:
                nb = -(-rows // 16)
                want = (nb, rows // nb)
            assert bench.prof.jit_blocks(k, rows) == want, (k, rows)
    assert bench.prof.jit_blocks(41, 20) == (2, 10)


def test_line_extras_cpu_baseline_on_every_rank0_line():
    """VERDICT r2 'next' 1: every N > 1 line carries the CPU baseline (rank 0,
    after the timed region); only rank 0 prints, and the heavy extras stay at
    world size 1 where no other rank waits at the closing barrier."""
    bench = load_bench()
    for config in (2, 3, 4, 5, 6, 7):
        for world in (2, 4, 8):
            ex = bench.line_extras(0, world, False, config)
            assert ex == {"cpu_baseline"}, (config, world, ex)
            for r in range(1, world):
                assert bench.line_extras(r, world, False, config) == set()
        one = bench.line_extras(0, 1, False, config)
        assert {"cpu_baseline", "traffic", "copy_ceiling"} <= one
        assert bench.line_extras(0, 1, True, config) == set()  # --minimal (PMC child runs)
    assert {"cpu_threads", "host_path", "shim_path"} <= bench.line_extras(0, 1, False, 2)


def test_bench_sets_dmabuf_ipc_before_torch():
    """RCCL ranks started by torch.distributed.run need
    HSA_ENABLE_IPC_MODE_LEGACY=0 before HIP loads: bench.py sets it ahead of
    `import torch`."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    i_env = src.index('os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")')
    i_torch = src.index("import torch")
    assert i_env < i_torch


def test_force_pg_flag_parses():
    bench = load_bench()
    a = bench.parse(["--force-pg", "--dist-backend", "nccl"])
    assert a.force_pg and a.dist_backend == "nccl"
    assert not bench.parse([]).force_pg


def test_all_rank_host_leg_policy():
    """the concurrent host-inclusive leg runs on EVERY
    rank at every world size for the host-bound geometries (the driver's
    1/2/4/8-GPU lines carry it), never in the PMC child runs."""
    bench = load_bench()
    for config in (2, 5, 6):
        assert bench.all_rank_leg(False, config, False)
        assert not bench.all_rank_leg(True, config, False)   # --minimal
        assert not bench.all_rank_leg(False, config, True)   # --no-host-path
    for config in (3, 4, 7):
        assert not bench.all_rank_leg(False, config, False)
    a = bench.parse([])
    assert a.pin == "numa" and a.host_mib == 256


def test_aggregate_all_ranks_is_sum_over_slowest():
    from benchkit import GIB, host
    recs = []
    for r, slow in ((0, 1.0), (1, 2.0)):
        geo = {}
        for name, chunk in host.ALL_RANK_GEOMETRIES:
            row = {"k": 4, "m_total": 6, "chunk_bytes": chunk, "chunks": 4, "lost": [0, 1],
                   "reps": 2, "bytes_per_rep": 4 * chunk, "roundtrip_pageable": True,
                   "roundtrip_pinned": True, "parity_modes_agree": True,
                   "parity_sha256": f"d{r}"}
            for leg in ("encode_pageable", "encode_pinned", "decode_pageable", "decode_pinned"):
                row[f"{leg}_s"] = slow
            geo[name] = row
        recs.append({"rank": r, "device": 0, "geometries": geo})
    pins = [{"gpu_numa_node": 0, "cpus": "0-7", "pinned": True}] * 2
    out = host.aggregate_all_ranks(recs, pins)
    assert out["ranks"] == 2
    for name, chunk in host.ALL_RANK_GEOMETRIES:
        g = out["geometries"][name]
        want = 2 * (2 * 4 * chunk) / GIB / 2.0
        assert abs(g["encode_pageable"]["aggregate_GiBps"] - round(want, 3)) < 1e-9
        assert g["encode_pageable"]["per_rank_GiBps"][0] == 2 * g["encode_pageable"]["per_rank_GiBps"][1]
        assert g["bit_exact"] and g["parity_sha256_per_rank"] == ["d0", "d1"]
    assert [p["cpus"] for p in out["per_rank"]] == ["0-7", "0-7"]


def test_cpu_ranges_and_pin_without_gpu():
    from benchkit import cpu
    assert cpu.cpu_ranges([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8"
    assert cpu.cpu_ranges([]) == ""
    saved = os.sched_getaffinity(0)
    info = cpu.pin_rank(0, "numa")  # no GPU here: node unknown, nothing pinned
    assert info["gpu_numa_node"] == -1 and not info["pinned"]
    assert os.sched_getaffinity(0) == saved
    with cpu.affinity(sorted(saved)[:1]):
        assert os.sched_getaffinity(0) == set(sorted(saved)[:1])
    assert os.sched_getaffinity(0) == saved
