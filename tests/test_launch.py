"""bench.py's rank launcher (storb_amd/launch.py) on CPU: the plan it takes
from --gpus and the environment, the rank processes it spawns (gloo, world
size 2 and 3, real rendezvous on 127.0.0.1), and the refusals that keep a
scaling line from silently being a 1-rank number."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

from storb_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_single_rank_default():
    p = launch.plan_launch(1, {}, device_count=1)
    assert (p.action, p.world, p.rank, p.device) == ("run", 1, 0, 0)


def test_plan_spawns_without_world_size():
    p = launch.plan_launch(8, {}, device_count=8)
    assert (p.action, p.world) == ("spawn", 8)


def test_plan_under_torchrun():
    env = {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}
    p = launch.plan_launch(4, env, device_count=8)
    assert (p.action, p.world, p.rank, p.device) == ("run", 4, 3, 3)


def test_plan_refuses_mismatch():
    with pytest.raises(SystemExit) as e:
        launch.plan_launch(8, {"WORLD_SIZE": "1", "RANK": "0"}, device_count=8)
    assert "disagrees" in str(e.value)
    with pytest.raises(SystemExit):
        launch.plan_launch(1, {"WORLD_SIZE": "2", "RANK": "0"}, device_count=8)


def test_plan_refuses_more_ranks_than_gpus_with_rccl():
    with pytest.raises(SystemExit) as e:
        launch.plan_launch(8, {}, device_count=1, dist_backend="nccl")
    assert "8 GPUs" in str(e.value)
    # the one-GPU rehearsal: every rank pinned to GPU 0, gloo
    p = launch.plan_launch(2, {"STORB_BENCH_DEVICE": "0"}, device_count=1,
                           dist_backend="gloo")
    assert (p.action, p.world) == ("spawn", 2)
    p = launch.plan_launch(2, {"STORB_BENCH_DEVICE": "0", "WORLD_SIZE": "2", "RANK": "1",
                               "LOCAL_RANK": "1"}, device_count=1, dist_backend="gloo")
    assert (p.rank, p.device) == (1, 0)


def test_plan_refuses_bad_counts():
    with pytest.raises(SystemExit):
        launch.plan_launch(0, {}, device_count=1)
    with pytest.raises(SystemExit):
        launch.plan_launch(2, {"WORLD_SIZE": "2", "RANK": "2"}, device_count=2)


def test_rank_env_is_torchrun_shaped():
    env = launch.rank_env({"X": "1"}, 1, 4, 29500)
    assert env["RANK"] == env["LOCAL_RANK"] == "1"
    assert env["WORLD_SIZE"] == "4" and env["MASTER_ADDR"] == "127.0.0.1"
    assert env["MASTER_PORT"] == "29500" and env["X"] == "1"


RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    sys.path.insert(0, {root!r})
    from storb_amd import launch
    plan = launch.plan_launch(int(sys.argv[1]), os.environ, 0, "gloo")
    assert plan.action == "run", plan
    dist.init_process_group("gloo")
    t = torch.tensor([float(plan.rank + 1)])
    dist.all_reduce(t)
    ranks = [None] * plan.world
    dist.all_gather_object(ranks, plan.rank)
    if plan.rank == 0:
        print(json.dumps({{"world": dist.get_world_size(), "sum": t.item(), "ranks": ranks}}),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(int(sys.argv[2]) if len(sys.argv) > 2 and plan.rank == 1 else 0)
""")


def _run_launcher(tmp_path, world, fail=None):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT.format(root=ROOT))
    extra = [] if fail is None else [str(fail)]
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {ROOT!r})
        from storb_amd import launch
        sys.exit(launch.spawn_ranks([{str(script)!r}, "{world}", *{extra!r}], {world},
                                    timeout=120))
    """)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=180, env=env)


@pytest.mark.parametrize("world", [2, 3])
def test_spawn_ranks_gloo(tmp_path, world):
    r = _run_launcher(tmp_path, world)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["world"] == world
    assert line["sum"] == world * (world + 1) / 2
    assert line["ranks"] == list(range(world))


def test_spawn_ranks_propagates_failure(tmp_path):
    r = _run_launcher(tmp_path, 2, fail=3)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    assert "disagrees with WORLD_SIZE" in r.stderr
