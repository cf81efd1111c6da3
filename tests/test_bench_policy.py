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


def test_jit_blocks_match_row_split_and_row_blocks(monkeypatch):
    bench = load_bench()
    monkeypatch.delenv("STORB_RS_JIT_SPLIT", raising=False)
    for k in (8, 12, 16, 17, 24, 40, 41, 63, 64):
        for rows in range(1, 33):
            if k % 2 == 0 and 16 < rows <= 32:
                want = (1, rows)
            else:
                nb = -(-rows // 16)
                want = (nb, rows // nb)
            assert bench.jit_blocks(k, rows) == want, (k, rows)
    monkeypatch.setenv("STORB_RS_JIT_SPLIT", "0")
    assert bench.jit_blocks(64, 32) == (2, 16)
    assert bench.jit_blocks(64, 20) == (2, 10)
