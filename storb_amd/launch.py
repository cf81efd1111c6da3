"""Rank launcher for the multi-GPU bench (BASELINE metric
"at 1/2/4/8 GPUs").

Storb's erasure stage partitions across GPUs without exchange: object i on
rank i mod N (upload.rs:418-420 / download.rs:505-529 run every object's
chunks independently). `bench.py --gpus N` therefore needs N processes, one
per GPU. Two ways in:

* under `torch.distributed.run` (the driver's form): RANK / LOCAL_RANK /
  WORLD_SIZE come from the environment and must agree with --gpus;
* plain `python bench.py --gpus N`: the parent spawns N rank processes of the
  same script *before any GPU call* (child processes, never an exec -- see
  the repo notes on exec after GPU init), waits for all of them and exits
  with the worst exit code.

Nothing here touches the GPU: `torch.cuda.device_count()` is the only probe
and it does not initialise HIP on this image.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import Mapping, Optional, Sequence


class LaunchError(SystemExit):
    """Inconsistent launch request; exits non-zero with the message."""

    def __init__(self, msg: str):
        super().__init__(f"bench launch: {msg}")


@dataclass(frozen=True)
class Plan:
    """What this process does: 'spawn' N rank children, or 'run' as one rank."""
    action: str          # "spawn" | "run"
    world: int
    rank: int = 0
    local_rank: int = 0
    device: int = 0      # GPU this rank uses


def plan_launch(gpus: int, env: Mapping[str, str], device_count: int,
                dist_backend: str = "nccl") -> Plan:
    """Decide from --gpus and the environment what this process is.

    * WORLD_SIZE set (torchrun or our own children): run as that rank; --gpus
      must equal WORLD_SIZE (a mismatch would mislabel a scaling line).
    * WORLD_SIZE unset, --gpus 1: run as the single rank.
    * WORLD_SIZE unset, --gpus N > 1: spawn N ranks.
    The device is LOCAL_RANK, or STORB_BENCH_DEVICE for every rank (the
    multi-rank rehearsal on a one-GPU box, gloo only). Each rank needs its own
    GPU with RCCL, so N > device_count is refused there.
    """
    if gpus < 1:
        raise LaunchError(f"--gpus must be >= 1 (got {gpus})")
    pinned = env.get("STORB_BENCH_DEVICE")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise LaunchError(f"--gpus {gpus} disagrees with WORLD_SIZE={world}")
        rank = int(env.get("RANK", "0"))
        local = int(env.get("LOCAL_RANK", str(rank)))
        if not 0 <= rank < world:
            raise LaunchError(f"RANK={rank} outside WORLD_SIZE={world}")
        action = "run"
    else:
        world, rank, local = gpus, 0, 0
        action = "spawn" if gpus > 1 else "run"
    device = int(pinned) if pinned is not None else local
    if pinned is None and world > 1 and dist_backend == "nccl" and world > device_count:
        raise LaunchError(f"{world} ranks need {world} GPUs, {device_count} visible")
    if action == "run" and device_count and device >= device_count:
        raise LaunchError(f"rank {rank} wants GPU {device}, {device_count} visible")
    return Plan(action, world, rank, local, device)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(base: Mapping[str, str], rank: int, world: int, port: int) -> dict:
    """The torch.distributed.run variables for rank `rank` of `world` on one
    node (rendezvous on 127.0.0.1: the container hostname may not resolve)."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    # dmabuf IPC is the only kind the host driver supports (RCCL needs it)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(argv: Sequence[str], world: int, env: Optional[Mapping[str, str]] = None,
                port: Optional[int] = None, timeout: Optional[float] = None) -> int:
    """Run `python argv...` as `world` rank processes; returns the worst exit
    code (first non-zero by rank order, or 0). If one rank fails the others
    are given a few seconds and then terminated, so a dead rendezvous cannot
    hang the launch."""
    base = dict(os.environ if env is None else env)
    port = port or free_port()
    procs = [subprocess.Popen([sys.executable, *argv], env=rank_env(base, r, world, port))
             for r in range(world)]
    t0 = time.monotonic()
    codes: list[Optional[int]] = [None] * world
    failed_at = None
    while any(c is None for c in codes):
        for r, p in enumerate(procs):
            if codes[r] is None:
                codes[r] = p.poll()
                if codes[r] not in (None, 0) and failed_at is None:
                    failed_at = time.monotonic()
        now = time.monotonic()
        if (failed_at is not None and now - failed_at > 20) or \
                (timeout is not None and now - t0 > timeout):
            for r, p in enumerate(procs):
                if codes[r] is None:
                    p.terminate()
            for r, p in enumerate(procs):
                if codes[r] is None:
                    try:
                        codes[r] = p.wait(timeout=10)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[r] = p.wait()
            break
        time.sleep(0.05)
    for c in codes:
        if c:
            return c if c > 0 else 128 - c
    return 0
