"""N > 1 bench path on the CPU (gloo, world sizes 2 and 3): each rank plans
its own shard of independent frames (config 5) with no data exchange, and
only the timing max and the parity AND cross ranks — the same helpers and the
same gloo group bench.py uses on the GPU node (it opens no RCCL communicator:
the barrier and the reductions are a few bytes on the host)."""
import json
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
torch = pytest.importorskip("torch")
dist = pytest.importorskip("torch.distributed")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as d
    import bench
    d.init_process_group("gloo", rank=rank, world_size=world)
    seed, gkey, desc = bench.shard_plan("c3", rank, world)
    elapsed = 1.0 + rank  # rank 1 is the slow one
    t = bench.max_over_ranks(d, torch, elapsed, "cpu")
    ok_all = bench.all_ranks(d, torch, True, "cpu")
    ok_one_bad = bench.all_ranks(d, torch, rank == 0, "cpu")
    d.barrier()
    d.destroy_process_group()
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(dict(seed=seed, gkey=gkey, desc=desc, t=t, ok_all=ok_all, ok_one_bad=ok_one_bad), f)


def test_two_rank_gloo_shards_and_reductions(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    cfgs = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))["configs"]
    for r, x in enumerate(res):
        assert x["seed"] == 0x5EED0005 + r
        assert x["gkey"] == f"c5_shard{r}" and x["gkey"] in cfgs
        assert x["t"] == 2.0                      # max over ranks
        assert x["ok_all"] is True and x["ok_one_bad"] is False
    assert res[0]["seed"] != res[1]["seed"]       # disjoint shards, no shared data


def test_single_rank_plan_is_config3():
    sys.path.insert(0, ROOT)
    import bench
    seed, gkey, _ = bench.shard_plan("c3", 0, 1)
    assert (seed, gkey) == (0x5EED0003, "c3_bin_64k")
    assert bench.max_over_ranks(None, torch, 3.5, "cpu") == 3.5


def test_bench_gpus2_launches_two_ranks_dry_run():
    """`bench.py --gpus 2` without a launcher starts 2 ranks itself
    (torch.distributed.run child process); --dry-run plans them on the CPU
    (gloo): rank 0 reports n_gpus = 2 and two disjoint shard plans."""
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["dry_run"] is True and out["n_gpus"] == 2
    seeds = sorted(p["seed"] for p in out["shards"])
    assert seeds == [0x5EED0005, 0x5EED0006]
    assert sorted(p["golden"] for p in out["shards"]) == ["c5_shard0", "c5_shard1"]
    assert out["max_elapsed"] == 2.0


@pytest.mark.parametrize("cfg,world", [("c4", 2), ("c3", 3)])
def test_bench_shard_one_batch_dry_run(cfg, world):
    """`bench.py --gpus N --shard-one-batch --dry-run`: ONE batch (config 4's
    irregular frames, or config 3) cut for N ranks by xyws_shard_plan_frames
    over the generator's table: every rank computes the same plan, the ranges
    tile the batch, start at frames, are balanced within one frame and carry
    the batch's whole payload. (The cut decoding to the unsplit bytes:
    tests/test_shard.py with the oracle; on the GPU, bench.py's parity.)"""
    import subprocess
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    from xynet_amd import _lib
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dry-run",
                        "--shard-one-batch", "--config", cfg], capture_output=True, text=True, timeout=300, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == world and len(out["shards"]) == world
    bounds = out["shards"][0]["bounds"]
    assert all(p["bounds"] == bounds for p in out["shards"])
    _, n, size, plens, offs = bench.generator_frames(_lib.load_tools(), cfg)
    assert bounds[0] == 0 and bounds[-1] == size and bounds == sorted(bounds)
    starts = set(offs.tolist())
    sizes = np.diff(np.append(offs, size))
    for k in range(1, world):
        assert bounds[k] in starts
        t = size * k // world
        i = int(np.searchsorted(offs, t, side="right")) - 1  # the frame holding the target
        assert abs(bounds[k] - t) <= sizes[i]
    assert sum(p["payload"] for p in out["shards"]) == int(plens.sum())
