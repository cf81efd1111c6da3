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
            assert bench.jit_blocks(k, rows) == want, (k, rows)
    assert bench.jit_blocks(41, 20) == (2, 10)


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
