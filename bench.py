#!/usr/bin/env python3
"""bench.py — device-resident WebSocket unmask throughput on MI355X.

Metric (BASELINE.json): GiB/s of payload decoded (header parse + boundary
discovery + in-place XOR unmask) per second, device resident, 64 KiB frames.

Workload per rank:
  N = 1 : config 3  — 32768 masked binary frames x 64 KiB payload (H = 14), one
          contiguous 2,147,942,400-byte batch, seed 0x5EED0003.
  N > 1 : config 5  — rank g decodes its own config-3-sized shard (seed
          0x5EED0005 + g) on its own GPU; frames are independent, so there is
          no data-path collective (weak scaling). Only the timing barrier and the
          max-over-ranks reduction use torch.distributed.
A step = one xyws_decode_stream call over the whole batch (boundaries found on
the device, every payload unmasked in place). XOR is an involution and headers
are never modified, so consecutive steps re-mask/unmask the same batch; the
parity check after the timed region compares the device digest with the
reference digest for that parity of step count (tests/golden/configs.json).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c1|c4]
                       [--mode fused|serial] [--no-cpu] [--host-path]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident WebSocket XOR-unmask, 64KiB frames, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
GIB = float(1 << 30)

CONFIGS = {
    # name: (nframes, payload, b0, seed, golden key, description)
    "c3": (32768, 65536, 0x82, 0x5EED0003, "c3_bin_64k",
           "config 3: 32768 x 64 KiB masked binary frames (H=14), one contiguous 2 GiB batch"),
    "c2": (1 << 20, 256, 0x82, 0x5EED0002, "c2_bin_256",
           "config 2: 2^20 x 256 B masked binary frames (H=8), one contiguous 264 MiB batch"),
    "c1": (65536, 4096, 0x81, 0x5EED0001, "c1_text_4k",
           "config 1 (device form): 65536 x 4 KiB masked text frames (H=8)"),
    "c4": (None, 1 << 30, None, 0x5EED0004, "c4_mixed",
           "config 4: mixed 1 B-1 MiB payloads, FIN=0 fragments + pings, >= 1 GiB batch"),
}


def hdr_len(p):
    return 2 + (0 if p < 126 else (2 if p <= 0xFFFF else 8)) + 4


def load_golden():
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        return json.load(f)["configs"]


def shard_plan(cfg_name, rank, world):
    """(seed, golden key, description) of this rank's batch. N > 1 on the
    64 KiB config is config 5: rank g owns its own config-3-sized shard of
    independent frames (seed 0x5EED0005 + g), so no rank needs another's data."""
    nframes, payload, b0, seed, gkey, desc = CONFIGS[cfg_name]
    if cfg_name == "c3" and world > 1:
        seed, gkey = 0x5EED0005 + rank, f"c5_shard{rank}"
        desc = ("config 5 shard: 32768 x 64 KiB masked binary frames (H=14), one contiguous 2 GiB "
                "batch per GPU, seed 0x5EED0005+rank")
    return seed, gkey, desc


def max_over_ranks(dist, torch, x, device):
    """The slowest rank's value (the job's elapsed time); x itself at N = 1."""
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks(dist, torch, ok, device):
    """True only if every rank's flag is true (parity of every shard)."""
    if dist is None:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def build_batch(torch, T, cfg_name, rank, world):
    """Generate this rank's batch in HBM; returns (buf, info)."""
    nframes, payload, b0, _, _, _ = CONFIGS[cfg_name]
    seed, gkey, desc = shard_plan(cfg_name, rank, world)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if nframes is not None:
        size = nframes * (hdr_len(payload) + payload)
        buf = torch.empty(size, dtype=torch.uint8, device="cuda")
        assert T.xyws_tools_fill_uniform(C.c_void_p(buf.data_ptr()), nframes, payload, b0, seed,
                                         stream) == 0
        payload_bytes = nframes * payload
        algo_bytes = nframes * (hdr_len(payload) + payload) + nframes * payload
    else:
        tot = C.c_uint64()
        n = T.xyws_tools_mixed_table(seed, payload, None, 0, C.byref(tot))
        tab = torch.empty(n * 32, dtype=torch.uint8)
        T.xyws_tools_mixed_table(seed, payload, C.c_void_p(tab.data_ptr()), n, C.byref(tot))
        import numpy as np
        rec = np.frombuffer(tab.numpy().tobytes(), dtype=np.dtype(
            [("off", "<u8"), ("plen", "<u8"), ("draw", "<u8"), ("b0", "u1"), ("hlen", "u1"),
             ("pad", "u1", 6)]))
        size = tot.value
        buf = torch.empty(size, dtype=torch.uint8, device="cuda")
        dtab = tab.cuda()
        assert T.xyws_tools_fill_mixed(C.c_void_p(buf.data_ptr()), size, C.c_void_p(dtab.data_ptr()),
                                       n, seed, stream) == 0
        nframes = n
        payload_bytes = int(rec["plen"].sum())
        algo_bytes = size + payload_bytes
    torch.cuda.synchronize()
    return buf, dict(nframes=nframes, payload_bytes=payload_bytes, algo_bytes=algo_bytes,
                     size=buf.numel(), golden=gkey, desc=desc, seed=seed)


def device_digest(torch, T, buf):
    out = torch.zeros(2, dtype=torch.int64, device=buf.device)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert T.xyws_tools_digest(C.c_void_p(buf.data_ptr()), buf.numel(), C.c_void_p(out.data_ptr()),
                               C.c_void_p(out.data_ptr() + 8), s) == 0
    return int(out[0].item()) & ((1 << 64) - 1)


def cpu_baseline(torch, buf, info, budget_s=12.0):
    """Time the reference CPU path (oracle/_ref: the reference headers compiled
    here) on a bounded host sample of the same batch. Returns a dict or None."""
    try:
        from oracle.oracle import Reference, Oracle, ref_lib_path
    except Exception as e:  # pragma: no cover
        return {"error": f"oracle import failed: {e}"}
    import numpy as np
    nframes, size = info["nframes"], info["size"]
    frame_bytes = size // max(nframes, 1)
    sample_frames = max(1, min(nframes, (512 << 20) // max(frame_bytes, 1)))
    sample_bytes = sample_frames * frame_bytes if info["golden"] != "c4_mixed" else min(size, 512 << 20)
    host = buf[:sample_bytes].cpu().numpy().copy()
    threads = max(1, min(16, os.cpu_count() or 1))
    kind = "reference" if os.path.exists(ref_lib_path("O2")) else "port"
    res = {"kind": kind, "unit": "GiB/s",
           "sample": f"first {sample_bytes} B of this rank's batch (host copy), whole frames only; "
                     f"{'reference headers compiled -O2 (oracle/_ref)' if kind == 'reference' else 'oracle C restatement -O2'}"}

    def run(fn, nbytes_payload, budget):
        reps, t0 = 0, time.perf_counter()
        while True:
            fn()
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return reps * nbytes_payload / dt / GIB

    payload_sample = sample_frames * (info["payload_bytes"] // max(nframes, 1))
    if kind == "reference":
        R = Reference("O2")
        res["value"] = run(lambda: R.decode_batch_mt(host, threads), payload_sample, budget_s / 2)
        res["cores"] = threads
        res["value_1core"] = run(lambda: R.decode_batch_mt(host, 1), payload_sample, budget_s / 2)
        try:
            R0 = Reference("O0")
            small = host[: max(frame_bytes, min(host.size, 32 << 20) // frame_bytes * frame_bytes)].copy()
            pay_small = (small.size // frame_bytes) * (info["payload_bytes"] // max(nframes, 1))
            res["value_O0_1core"] = run(lambda: R0.decode_batch_mt(small, 1), pay_small, 2.0)
        except Exception:
            pass
    else:
        O = Oracle()
        res["value"] = run(lambda: O.decode_stream(host, cap=16), payload_sample, budget_s)
        res["cores"] = 1
    return res


def host_path_rate(torch, ws, info, buf, chunk=256 << 20, reps=3):
    """PCIe-inclusive rate for DESIGN.md: pinned host batch -> H2D -> decode -> D2H,
    chunked over 3 streams (not the bench value)."""
    size = buf.numel()
    hostbuf = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    hostbuf.copy_(buf.cpu())
    streams = [torch.cuda.Stream() for _ in range(3)]
    devs = [torch.empty(chunk + (1 << 20), dtype=torch.uint8, device="cuda") for _ in range(3)]
    decs = [ws.frame_decoder() for _ in range(3)]
    # chunks cut at frame boundaries of the uniform batch (carry not needed)
    fb = size // info["nframes"]
    per = max(1, chunk // fb) * fb
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for i, off in enumerate(range(0, size, per)):
            k = i % 3
            n = min(per, size - off)
            with torch.cuda.stream(streams[k]):
                d = devs[k][:n]
                d.copy_(hostbuf[off:off + n], non_blocking=True)
                decs[k].decode(d, cap=0, count=False, carry=False)
                hostbuf[off:off + n].copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return reps * info["payload_bytes"] / dt / GIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="fused", choices=["fused", "serial"])
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--host-path", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--stats", action="store_true", help="print fused-decoder resolution counters")
    ap.add_argument("--xopts", type=lambda x: int(x, 0), default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from xynet_amd import _lib, websocket as ws
    T = _lib.load_tools()
    buf, info = build_batch(torch, T, args.config, rank, world)
    golden = load_golden().get(info["golden"])
    dec = ws.frame_decoder(serial=(args.mode == "serial"))
    dec.opts |= args.xopts
    dec.ctx.reserve(buf.numel(), 0)
    stream = torch.cuda.current_stream()

    def step():  # fresh stream each step: no carry in/out, no frame table, no count
        dec.decode(buf, cap=0, count=False, carry=False)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        dec.decode(buf, cap=0, count=False, carry=False)
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = max_over_ranks(dist, torch, t1 - t0, "cuda")
    kernel_ms = sorted(a.elapsed_time(b) for a, b in evs)
    avg_ms = sum(kernel_ms) / len(kernel_ms)

    if args.stats and rank == 0:  # one extra counted decode pair (keeps the step parity)
        names = ["runs", "runs_without_entry", "bad_boundaries", "repairs", "cuts", "spins", "dense_passes",
                 "frames", "scan_segments", "scan_survivors", "scan_undecided", "cyc_scan_filter",
                 "cyc_scan_check", "cyc_scan_resolve", "cyc_dense_entry", "cyc_dense_chase", "cyc_prologue", "cyc_main", "cyc_wait",
                 "cyc_fill", "cyc_chase_sync", "cyc_xor", "cyc_tail", "cyc_prefetch_issue", "cyc_chase_pass",
                 "cyc_pro_fill", "cyc_pro_scan", "cyc_pro_publish", "dense_no_entry", "dense_chase_fail",
                 "dense_mismatch", "dense_overflow", "giveups", "bridges", "-"]
        for _ in range(2):
            dec.opts |= _lib.OPT_STATS
            dec.decode(buf, cap=0, count=False, carry=False)
            dec.opts &= ~_lib.OPT_STATS
            out = (C.c_uint64 * _lib.NSTATS)()
            dec.ctx.L.xyws_debug_stats(dec.ctx.h, C.c_void_p(stream.cuda_stream), out)
        st = {k: v for k, v in zip(names, list(out)) if k != "-"}
        nrun = max(1, st["runs"] + 1)
        for k in list(st):
            if k.startswith("cyc_"):
                st[k.replace("cyc_", "us_per_run_")] = round(st.pop(k) / nrun / 2100.0, 3)
        print(json.dumps({"stats": st}), flush=True)

    # parity after the timed region: total decodes = warmup + steps
    dev_err = dec.ctx.last_device_error()
    dig = device_digest(torch, T, buf)
    odd = (args.warmup + args.steps) % 2 == 1
    parity = None
    if golden is not None:
        parity = (dig == (golden["out_digest"] if odd else golden["in_digest"])) and dev_err == 0

    total_payload = info["payload_bytes"] * world
    value = args.steps * total_payload / elapsed / GIB
    achieved = info["algo_bytes"] / (avg_ms * 1e-3) / 1e9

    parities = [all_ranks(dist, torch, parity, "cuda") if dist else parity]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # sample taken from a masked-state batch: regenerate if an odd count was applied
        if odd:
            step()
            torch.cuda.synchronize()
        cpu = cpu_baseline(torch, buf, info, args.cpu_budget)
        if odd:
            step()
            torch.cuda.synchronize()
    host_rate = None
    if args.host_path and rank == 0 and info["nframes"] and args.config != "c4":
        host_rate = host_path_rate(torch, ws, info, buf)

    traffic = None
    pmc_file = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_file):
        try:
            pm = json.load(open(pmc_file))
            rec = pm.get(args.config + ":" + args.mode)
            if rec:
                traffic = rec["hbm_bytes_per_launch"]
        except Exception:
            traffic = None

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 masked frames generated in HBM; include/xyws_synth.h)",
            "config": {
                "workload": info["desc"],
                "mode": args.mode + " (xyws_decode_stream: boundaries discovered on device)",
                "frames_per_gpu": info["nframes"],
                "batch_bytes_per_gpu": info["size"],
                "payload_bytes_per_gpu": info["payload_bytes"],
                "parallelism": f"shard-by-frame x{world}, no collective",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": info["algo_bytes"],
                "kernel_ms_avg": round(avg_ms, 4),
                "kernel_ms_min": round(kernel_ms[0], 4),
            },
            "cpu_baseline": cpu,
            "parity": bool(parities[0]) if parities[0] is not None else None,
        }
        if host_rate is not None:
            line["host_path_gibs"] = round(host_rate, 3)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
