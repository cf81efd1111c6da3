"""Who runs the bench line: each rank's GPU and process-group view
(rank_info), which bounded extras a rank adds after the timed region
(line_extras, all_rank_leg), and the one process group per job (init_pg).
See storb_amd/launch.py for how the rank processes start."""
from __future__ import annotations

import os
import platform

import torch
import torch.distributed as dist

from storb_amd import launch


def rank_info(rank, world, local, dev, use_pg):
    """Who ran: every rank's GPU (ordinal + PCI bus) and the process group's
    own rank count, so a scaling line cannot silently be a 1-rank number."""
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "device": local, "name": props.name,
          "pci_bus": getattr(props, "pci_bus_id", None), "host": platform.node()}
    if not use_pg:
        return {"world_size": 1, "backend": None, "pg_ranks": 1, "ranks": [me]}
    ranks = [None] * world
    dist.all_gather_object(ranks, me)
    return {"world_size": world, "backend": dist.get_backend(),
            "pg_ranks": dist.get_world_size(), "ranks": ranks,
            "distinct_gpus": len({(r["host"], r["device"]) for r in ranks})}


def line_extras(rank, world, minimal, config):
    """The bounded, untimed extras this rank adds to its line, all run after
    the last barrier of the timed region. Rank 0 always carries the
    single-thread CPU baseline (N > 1 lines too: the driver's scaling lines
    need it beside the GPU figure); the heavier ones (live PMC traffic passes,
    copy ceiling, threaded CPU baselines, PCIe-inclusive and per-call host
    rates, hashing, repair) only at world size 1, where no other rank waits."""
    if rank != 0 or minimal:
        return set()
    ex = {"cpu_baseline"}
    if world > 1:
        return ex
    ex |= {"traffic", "copy_ceiling", "kernel_trace"}
    if config in (2, 5, 6):
        ex |= {"cpu_threads", "host_path", "shim_path", "hashing", "repair", "download"}
    if config == 3:
        ex.add("assembly")
    if config == 4:
        ex.add("storb_faithful")
    return ex


def all_rank_leg(minimal, config, no_host_path):
    """Whether every rank runs the concurrent host-inclusive leg
    (benchkit/host.py all_ranks_host_leg) after the timed region: at every
    world size, so the driver's 1/2/4/8-GPU lines carry the host-side
    scaling limit of SURVEY 8(e) beside the device-resident value."""
    return not minimal and not no_host_path and config in (2, 5, 6)


def init_pg(a, world, dev):
    """One process group per job: RCCL ('nccl') with each rank bound to its
    GPU, or gloo for the rehearsal with several ranks on one GPU. --force-pg
    at world size 1 creates a one-rank group so the exact multi-rank sequence
    runs on a one-GPU box."""
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(launch.free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if a.dist_backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(a.dist_backend)
    if dist.get_world_size() != world:
        raise SystemExit(f"process group has {dist.get_world_size()} ranks, expected {world}")
