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
                       [--mode fused|serial] [--no-cpu] [--host-path] [--copies C] [--dry-run]
--gpus N without a launcher starts N ranks (torch.distributed.run, one process
per GPU) as a child process and passes their output through.
"""
import argparse
import ctypes as C
import json
import os
import sys
import statistics
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


def cpu_threads():
    """Host threads for the CPU baseline: the CPUs this process may run on
    (sched_getaffinity), capped by OMP_NUM_THREADS when set (the GPU box sets
    it to the box's CPU share; os.cpu_count() there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(torch, buf, info, budget_s=12.0):
    """Time the CPU path on a bounded host sample of the same batch.

    Primary (kind "port"): the committed C restatement of the reference hot
    path (oracle/xyws_oracle.c, pinned to the reference's golden vectors) at
    -O2 on all usable host threads: serial header walk + threaded unmask.
    Beside it: the same at 1 thread, at -O0 (as the reference builds,
    CMakeLists.txt:4), and the reference's own headers (oracle/_ref) when that
    container-built library is present."""
    try:
        from oracle.oracle import Oracle, Reference, ref_lib_path, oracle_lib_path
    except Exception as e:  # pragma: no cover
        return {"error": f"oracle import failed: {e}"}
    nframes, size = info["nframes"], info["size"]
    frame_bytes = size // max(nframes, 1)
    if info["golden"] == "c4_mixed":
        sample_bytes = min(size, 512 << 20)
        payload_sample = int(info["payload_bytes"] * sample_bytes / size)
    else:
        sample_frames = max(1, min(nframes, (512 << 20) // max(frame_bytes, 1)))
        sample_bytes = sample_frames * frame_bytes
        payload_sample = sample_frames * (info["payload_bytes"] // max(nframes, 1))
    host = buf[:sample_bytes].cpu().numpy().copy()
    threads = cpu_threads()

    def rate(fn, nbytes_payload, budget, samples=5):
        # the median of `samples` timed samples, each at least
        # one whole pass over the sample and about budget / samples long
        rates = []
        for _ in range(samples):
            reps, t0 = 0, time.perf_counter()
            while True:
                fn()
                reps += 1
                dt = time.perf_counter() - t0
                if dt >= budget / samples:
                    break
            rates.append(reps * nbytes_payload / dt / GIB)
        return round(statistics.median(rates), 4)

    small = host[: max(frame_bytes, min(host.size, 32 << 20) // max(frame_bytes, 1) * frame_bytes)].copy()
    pay_small = int(payload_sample * small.size / max(host.size, 1))
    O2 = Oracle()
    res = {"kind": "port", "unit": "GiB/s", "cores": threads, "nproc": os.cpu_count(),
           "cores_reason": "the CPUs this process may run on (sched_getaffinity), capped by OMP_NUM_THREADS "
                           f"({os.environ.get('OMP_NUM_THREADS', 'unset')}: the GPU box's CPU share; nproc shows "
                           "the whole machine)",
           "statistic": "median of 5 timed samples per figure",
           "sample": f"first {sample_bytes} B of this rank's batch (host copy, whole frames): "
                     f"oracle/xyws_oracle.c restatement -O2, serial header walk + unmask on {threads} threads",
           "value": rate(lambda: O2.decode_batch_mt(host, threads), payload_sample, budget_s * 0.4),
           "value_1core": rate(lambda: O2.decode_batch_mt(host, 1), payload_sample, budget_s * 0.2)}
    try:
        O0 = Oracle(oracle_lib_path("O0"))
        res["value_O0_1core"] = rate(lambda: O0.decode_batch_mt(small, 1), pay_small, budget_s * 0.1)
    except Exception:
        pass
    sha_file = os.path.join(os.path.dirname(ref_lib_path("O2")), "SOURCE_SHA")
    if os.path.exists(ref_lib_path("O2")) and not os.path.exists(sha_file):
        res["reference"] = {"dropped": "oracle/_ref has no SOURCE_SHA stamp (not built by oracle/Makefile)"}
    elif os.path.exists(ref_lib_path("O2")):  # the reference headers themselves (container-built)
        try:
            R = Reference("O2")
            ref = {"value": rate(lambda: R.decode_batch_mt(host, threads), payload_sample, budget_s * 0.2),
                   "cores": threads, "src_sha": open(sha_file).read().strip(),
                   "src_sha_of": "oracle/Makefile: websocket_frame_header.h, websocket_frame_mask.h, "
                                 "ref_harness.cpp, include/xyws.h"}
            if os.path.exists(ref_lib_path("O0")):
                R0 = Reference("O0")
                ref["value_O0_1core"] = rate(lambda: R0.decode_batch_mt(small, 1), pay_small, budget_s * 0.1)
            res["reference"] = ref
        except Exception:
            pass
    return res


def host_path_rate(torch, ws, T, info, buf, golden, chunk=256 << 20, reps=3, nstreams=3):
    """PCIe-inclusive rate for DESIGN.md (never the bench value): pinned host
    batch -> H2D -> decode -> D2H, chunked at frame boundaries over `nstreams`
    streams (one context: per-stream scratch). An odd number of passes leaves
    the host batch decoded; its digest and the device error word are checked."""
    size = buf.numel()
    hostbuf = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    hostbuf.copy_(buf.cpu())  # (buf holds the masked input batch)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    devs = [torch.empty(chunk + (1 << 20), dtype=torch.uint8, device="cuda") for _ in range(nstreams)]
    dec = ws.frame_decoder()
    fb = size // info["nframes"]
    per = max(1, chunk // fb) * fb
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for i, off in enumerate(range(0, size, per)):
            k = i % nstreams
            n = min(per, size - off)
            with torch.cuda.stream(streams[k]):
                d = devs[k][:n]
                d.copy_(hostbuf[off:off + n], non_blocking=True)
                dec.decode(d, cap=0, count=False, carry=False)
                hostbuf[off:off + n].copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    err = dec.ctx.last_device_error()
    # host digest of the result (odd reps: each chunk decoded an odd number of times)
    chk = torch.empty(size, dtype=torch.uint8, device="cuda")
    chk.copy_(hostbuf)
    dig = device_digest(torch, T, chk)
    want = golden["out_digest"] if reps % 2 == 1 else golden["in_digest"]
    return {"gibs": round(reps * info["payload_bytes"] / dt / GIB, 3), "streams": nstreams,
            "chunk_bytes": per, "passes": reps, "parity": dig == want and err == 0, "device_error": err}


def arena_path_rate(torch, ws, T, info, buf, golden, conns=4, recv=16 << 20):
    """PCIe-inclusive rate through the io_uring-facing API (xyws_arena_*, never
    the bench value): the batch split at frame boundaries over `conns`
    connections, each one's bytes in its own pinned arena, submitted in
    `recv`-byte pieces cut anywhere (the carry chains across them on the
    device), completions taken from one eventfd with poll() as an io_uring loop
    would. One pass: the arenas then hold the decoded batch (digest checked)."""
    import ctypes as C
    import select
    size = buf.numel()
    fb = size // info["nframes"]
    per = -(-info["nframes"] // conns) * fb
    fd = os.eventfd(0, os.EFD_NONBLOCK)
    arenas, plan = [], []
    for k, off in enumerate(range(0, size, per)):
        n = min(per, size - off)
        a = ws.RecvArena(n, max(1, n // fb + 2), eventfd=fd)
        view = torch.frombuffer((C.c_uint8 * n).from_address(a.host_ptr), dtype=torch.uint8)
        view.copy_(buf[off:off + n])  # (the masked input, D2H into the pinned arena)
        arenas.append((a, off, n, view))
        plan.append([(o, min(recv, n - o)) for o in range(0, n, recv)])
    torch.cuda.synchronize()
    poller = select.poll()
    poller.register(fd, select.POLLIN)
    pending = [[] for _ in arenas]
    nxt = [0] * len(arenas)
    t0 = time.perf_counter()
    while any(nxt[k] < len(plan[k]) or pending[k] for k in range(len(arenas))):
        progressed = False
        for k, (a, _, _, _) in enumerate(arenas):
            while nxt[k] < len(plan[k]):
                s = a.submit(*plan[k][nxt[k]])
                if s is None:
                    break
                pending[k].append(s)
                nxt[k] += 1
                progressed = True
            while pending[k] and a.poll(pending[k][0]) is not None:
                pending[k].pop(0)
                progressed = True
        if not progressed and poller.poll(1000):
            os.eventfd_read(fd)
    dt = time.perf_counter() - t0
    chk = torch.empty(size, dtype=torch.uint8, device="cuda")
    for a, off, n, view in arenas:
        chk[off:off + n].copy_(view)
    dig = device_digest(torch, T, chk)
    err = ws.context().last_device_error()
    for a, _, _, _ in arenas:
        a.close()
    os.close(fd)
    return {"gibs": round(info["payload_bytes"] / dt / GIB, 3), "connections": len(arenas), "recv_bytes": recv,
            "api": "xyws_arena_submit / eventfd", "parity": dig == golden["out_digest"] and err == 0,
            "device_error": err}


def copy_ceiling(torch, ws, buf, reps=10):
    """The same-box ceiling for this batch's traffic, measured in the run:
    (a) an in-place XOR of the whole batch with one key (xyws_unmask,
    k_unmask_range: every byte read and written once, no boundaries: the
    decode's traffic with nothing to resolve), (b) a D2D hipMemcpy of the batch
    into a scratch buffer (torch copy_). GB/s over `reps` launches each, HIP
    events; an even number of XOR passes leaves the batch as it was."""
    reps += reps % 2
    stream = torch.cuda.current_stream()
    ctx = ws.Context(buf.device.index or 0)
    key = (C.c_uint8 * 4)(0x5A, 0xC3, 0x96, 0x21)
    n = buf.numel()

    def xor_pass():
        assert ctx.L.xyws_unmask(ctx.h, C.c_void_p(buf.data_ptr()), n, key, 0, None,
                                 C.c_void_p(stream.cuda_stream)) == 0

    def timed(fn):
        fn()
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    ms_xor = timed(xor_pass)
    dst = torch.empty_like(buf)
    ms_cpy = timed(lambda: dst.copy_(buf))
    del dst
    return {"unmask_inplace_gbs": round(2 * n / (ms_xor * 1e-3) / 1e9, 1),
            "d2d_copy_gbs": round(2 * n / (ms_cpy * 1e-3) / 1e9, 1),
            "bytes_per_launch": 2 * n, "reps": reps,
            "what": "in-place XOR of the batch with one key (xyws_unmask) and D2D hipMemcpy of the batch, "
                    "same device, in this run: read + write bytes / HIP-event time"}


def source_hash():
    """Hash of the decoder sources, stamped on PMC records (profiles/pmc_traffic.json)
    so that a traffic figure is only reported for the kernel it was measured on."""
    import hashlib
    h = hashlib.sha256()
    for f in ("xyws_stream.hip", "xyws_device.h", "xyws_stream.h", "xyws.hip", "xyws_lattice.h"):
        with open(os.path.join(ROOT, "xynet_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(config, mode):
    """HBM bytes per decoder kernel launch from profiles/pmc_traffic.json when
    that record was measured on these exact decoder sources; else None."""
    pmc_file = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(pmc_file):
        return None, "no PMC record"
    try:
        rec = json.load(open(pmc_file)).get(config + ":" + mode)
    except Exception:
        return None, "unreadable PMC record"
    if not rec:
        return None, f"no PMC record for {config}:{mode}"
    if rec.get("src_sha") != source_hash():
        return None, f"PMC record {rec.get('src_sha')} is from other decoder sources ({source_hash()})"
    return rec["hbm_bytes_per_launch"], f"profiles/pmc_traffic.json {config}:{mode} ({rec.get('profile', '?')})"


# --op: the §8(f) callers on the decoded batch (tests/golden/gen_ops_golden.py
# holds the same parameters and writes the expected digests)
OP_PARAMS = {"enc_flags": 0x11, "cls_max_payload": 1 << 20, "cls_policy": 0x1, "rs_opts": 0x1}
OP_GOLDEN_KEYS = {"c1": "c1_text_4k", "c2": "c2_bin_256", "c3": "c3_bin_64k", "c4": "c4_mixed"}


def op_bench(args, torch, T, ws, info, buf):
    """One §8(f) caller timed over the decoded batch (not the headline):
    encode = echo_once's replies for every frame (xyws_encode_frames),
    classify = the close policy per frame (xyws_classify_frames), reassemble =
    FIN=0 chains into messages + UTF-8 (xyws_reassemble). The frame table comes
    from one untimed decode with descriptors. Algorithmic bytes per call: the
    descriptors read (32 B per frame) + payload bytes read + bytes written
    (replies / 8 B verdicts / gathered payload + 40 B message records)."""
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)
    ctx = ws.context()
    L, h = ctx.L, ctx.h
    nmax = info["nframes"] + 2
    frames_t = torch.empty(nmax * 32, dtype=torch.uint8, device="cuda")
    n_t = torch.zeros(1, dtype=torch.int64, device="cuda")
    assert L.xyws_decode_stream(h, C.c_void_p(buf.data_ptr()), buf.numel(), None, None,
                                C.c_void_p(frames_t.data_ptr()), nmax, C.c_void_p(n_t.data_ptr()), 0, sp) == 0
    torch.cuda.synchronize()
    nf = int(n_t.item())
    src, slen = C.c_void_p(buf.data_ptr()), buf.numel()
    fr = C.c_void_p(frames_t.data_ptr())
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "ops.json")))["configs"].get(
        OP_GOLDEN_KEYS.get(args.config), {})
    plen = int(frames_t[: nf * 32].view(torch.int64).view(-1, 4)[:, 2].sum().item())
    olen = torch.zeros(1, dtype=torch.int64, device="cuda")
    if args.op == "encode":
        assert L.xyws_encode_frames(h, src, slen, fr, nf, None, OP_PARAMS["enc_flags"], 0, None, None, 0, None, 0,
                                    None, C.c_void_p(olen.data_ptr()), sp) == 0
        torch.cuda.synchronize()
        total = int(olen.item())
        out = torch.empty(max(total, 1), dtype=torch.uint8, device="cuda")

        def step():
            assert L.xyws_encode_frames(h, src, slen, fr, nf, None, OP_PARAMS["enc_flags"], 0, None, None, 0,
                                        C.c_void_p(out.data_ptr()), total, None, C.c_void_p(olen.data_ptr()), sp) == 0
        algo = 32 * nf + plen + total

        def parity():
            g = gold.get("encode", {})
            return int(olen.item()) == g.get("out_len") and device_digest(torch, T, out[:total]) == g.get("out_digest")
        what = "echo replies (FIN|TEXT, unmasked) for every frame"
    elif args.op == "classify":
        verd = torch.zeros(max(nf, 1) * 8, dtype=torch.uint8, device="cuda")
        first = torch.zeros(1, dtype=torch.int64, device="cuda")

        def step():
            assert L.xyws_classify_frames(h, src, slen, fr, nf, None, OP_PARAMS["cls_max_payload"],
                                          OP_PARAMS["cls_policy"], C.c_void_p(verd.data_ptr()),
                                          C.c_void_p(first.data_ptr()), sp) == 0
        algo = 32 * nf + 8 * nf

        def parity():
            g = gold.get("classify", {})
            return (device_digest(torch, T, verd[: nf * 8]) == g.get("verdicts_digest") and
                    (int(first.item()) & ((1 << 64) - 1)) == g.get("first_close"))
        what = "close policy per frame (FRAGMENTS, max payload 1 MiB)"
    else:
        out = torch.empty(max(plen, 1), dtype=torch.uint8, device="cuda")
        msgs = torch.zeros(max(nf, 1) * 40, dtype=torch.uint8, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")

        def step():
            assert L.xyws_reassemble(h, src, slen, fr, nf, None, OP_PARAMS["rs_opts"], C.c_void_p(out.data_ptr()),
                                     plen, C.c_void_p(msgs.data_ptr()), nf, C.c_void_p(cnt.data_ptr()), sp) == 0
        algo = 32 * nf + 2 * plen + 40 * nf

        def parity():
            g = gold.get("reassemble", {})
            nm = int(cnt.item())
            return (nm == g.get("messages") and device_digest(torch, T, out[:plen]) == g.get("out_digest") and
                    device_digest(torch, T, msgs[: nm * 40]) == g.get("msgs_digest"))
        what = "FIN=0 chains into messages + UTF-8 validation"
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / args.steps
    ok = bool(gold) and parity() and ctx.last_device_error() == 0
    gbs = algo / (ms * 1e-3) / 1e9
    print(json.dumps({
        "metric": f"xyws {args.op} throughput (§8(f) caller, device-resident)", "op": args.op,
        "value": round(gbs, 1), "unit": "GB/s (algorithmic bytes)", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "dtype": "u8", "data": "synthetic, decoded by one untimed xyws_decode_stream",
        "config": {"workload": info["desc"], "op": what, "frames": nf, "payload_bytes": plen},
        "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_call": algo,
                     "kernel_ms_avg": round(ms, 4),
                     "note": "HIP-event time per call (all of the op's kernels and launch gaps)"},
        "parity": ok}), flush=True)


def launch_ranks(args):
    """--gpus N without a launcher: start N ranks with torch.distributed.run as
    a CHILD process (nothing in this parent touches the GPU), pass their output
    through, and exit with its status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def generator_frames(T, cfg_name):
    """Frame starts of a config's generated batch as host xyws_frame records
    (frame_off set), from the generator's own table: the host-side prefix
    over frame sizes at generation time. Returns (records
    as a ctypes array, n, batch bytes, payload bytes per frame)."""
    import numpy as np
    from xynet_amd import _lib
    nframes, payload, b0, seed, _, _ = CONFIGS[cfg_name]
    if nframes is not None:
        fb = hdr_len(payload) + payload
        offs = np.arange(nframes, dtype=np.int64) * fb
        plens = np.full(nframes, payload, dtype=np.int64)
        size = nframes * fb
    else:
        tot = C.c_uint64()
        n = T.xyws_tools_mixed_table(seed, payload, None, 0, C.byref(tot))
        tab = (C.c_uint8 * (32 * n))()
        T.xyws_tools_mixed_table(seed, payload, tab, n, C.byref(tot))
        rec = np.frombuffer(bytes(tab), dtype=np.dtype(
            [("off", "<u8"), ("plen", "<u8"), ("draw", "<u8"), ("b0", "u1"), ("hlen", "u1"), ("pad", "u1", 6)]))
        offs = rec["off"].astype(np.int64)
        plens = rec["plen"].astype(np.int64)
        size = int(tot.value)
    recs = np.zeros((offs.size, 4), dtype=np.int64)
    recs[:, 0] = offs
    recs[:, 2] = plens
    arr = (_lib.Frame * max(1, offs.size)).from_buffer_copy(recs.tobytes().ljust(32 * max(1, offs.size), b"\0"))
    return arr, int(offs.size), size, plens, offs


def one_batch_plan(T, cfg_name, world):
    """--shard-one-batch: ONE config batch cut into `world` frame-aligned,
    byte-balanced ranges (xyws_shard_plan_frames over the generator's table).
    Returns (bounds, payload bytes per shard)."""
    import numpy as np
    from xynet_amd import _lib
    arr, n, size, plens, offs = generator_frames(T, cfg_name)
    out = (C.c_uint64 * (world + 1))()
    rc = _lib.load().xyws_shard_plan_frames(arr, n, size, world, out)
    assert rc == 0, rc
    bounds = list(out)
    idx = np.searchsorted(offs, np.array(bounds[1:-1], dtype=np.int64))
    cuts = [0] + [int(i) for i in idx] + [n]
    pay = [int(plens[cuts[k]:cuts[k + 1]].sum()) for k in range(world)]
    return bounds, pay


def dry_run(world, rank, args):
    """--dry-run: the N-rank plan without a GPU (gloo): every rank plans its
    own shard; rank 0 prints the gathered plan (tests/test_multirank.py).
    With --shard-one-batch every rank plans the cut of the one batch."""
    import torch.distributed as dist
    dist.init_process_group("gloo")
    if args.shard_one_batch:
        from xynet_amd import _lib
        bounds, pay = one_batch_plan(_lib.load_tools(), args.config, world)
        plans = [None] * world
        dist.all_gather_object(plans, {"rank": rank, "bounds": bounds, "range": bounds[rank:rank + 2],
                                       "payload": pay[rank]})
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "one_batch": args.config, "shards": plans}),
                  flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return
    seed, gkey, desc = shard_plan("c3", rank, world)
    plans = [None] * world
    dist.all_gather_object(plans, {"rank": rank, "seed": seed, "golden": gkey})
    t = max_over_ranks(dist, __import__("torch"), 1.0 + rank, "cpu")
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "shards": plans, "max_elapsed": t}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="fused", choices=["fused", "serial"])
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the in-run copy-ceiling measurement")
    ap.add_argument("--host-path", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--copies", type=int, default=0,
                    help="batch copies rotated over the steps (0: enough to exceed the 256 MiB Infinity Cache)")
    ap.add_argument("--dry-run", action="store_true", help="plan the N-rank run on the CPU (gloo) and exit")
    ap.add_argument("--stats", action="store_true", help="print fused-decoder resolution counters")
    ap.add_argument("--frames", action="store_true",
                    help="every step also returns the whole frame table and count (not the headline)")
    ap.add_argument("--settle", type=int, default=30,
                    help="untimed decodes before the timed steps, counting the W warm-up steps (default 30)")
    ap.add_argument("--shard-one-batch", action="store_true",
                    help="N > 1: ONE config batch cut at frame boundaries across the ranks (xyws_shard_plan_frames; "
                         "strong scaling), instead of one independent shard per rank (config 5)")
    ap.add_argument("--op", default="decode", choices=["decode", "encode", "classify", "reassemble"],
                    help="time a §8(f) caller on the decoded batch instead of the decode (not the headline)")
    ap.add_argument("--xopts", type=lambda x: int(x, 0), default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(world, rank, args)

    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        # gloo (host TCP): the ranks share nothing on the data path — each
        # decodes its own frames in its own HBM — so the only cross-rank
        # traffic is the timing barrier, the max over ranks and the parity
        # AND, a few bytes on the host after torch.cuda.synchronize(); no RCCL
        # communicator is created
        import torch.distributed as dist
        dist.init_process_group("gloo")

    from xynet_amd import _lib, websocket as ws
    T = _lib.load_tools()
    one = args.shard_one_batch
    # --shard-one-batch: every rank holds the same (whole) batch and decodes
    # only its frame-aligned range of it; the others' ranges are decoded after
    # the timed region so that the whole batch's digest checks the cut
    buf0, info = build_batch(torch, T, args.config, 0 if one else rank, 1 if one else world)
    if args.op != "decode":
        return op_bench(args, torch, T, ws, info, buf0)
    golden = load_golden().get(info["golden"])
    bounds = None
    if one:
        bounds, pay = one_batch_plan(T, args.config, world)
        lo_b, hi_b = bounds[rank], bounds[rank + 1]
        info["whole_payload_bytes"] = info["payload_bytes"]
        info["payload_bytes"] = pay[rank]
        info["algo_bytes"] = (hi_b - lo_b) + pay[rank]
    # Batches below the 256 MiB Infinity Cache (c1, c2) are timed over >= 4
    # copies used in turn, so that each step reads its batch from HBM
    # (SURVEY.md §7); every copy's parity is checked.
    span = info["size"] if bounds is None else max(1, bounds[rank + 1] - bounds[rank])  # bytes one step reads
    ncopies = args.copies or (1 if span >= (1 << 30) else max(4, -(-(1 << 30) // span)))
    bufs = [buf0] + [buf0.clone() for _ in range(ncopies - 1)]
    uses = [0] * ncopies
    dec = ws.frame_decoder(serial=(args.mode == "serial"))
    dec.opts |= args.xopts
    dec.ctx.reserve(info["size"], 0)
    stream = torch.cuda.current_stream()

    # --frames: every step also returns the whole frame table and the count
    # (what a websocket_recv_data caller consumes), into buffers allocated once
    frames_t = n_t = None
    if args.frames:
        frames_t = torch.empty(max(1, info["nframes"] + 2) * 32, dtype=torch.uint8, device="cuda")
        n_t = torch.zeros(1, dtype=torch.int64, device="cuda")

    def part(b, r=rank):  # the range this rank decodes
        return b if bounds is None else b[bounds[r]:bounds[r + 1]]

    def step(i):  # fresh stream each step: no carry in/out (no frame table, no count by default)
        k = i % ncopies
        uses[k] += 1
        b = part(bufs[k])
        if frames_t is None:
            dec.decode(b, cap=0, count=False, carry=False)
            return
        rc = dec.ctx.L.xyws_decode_stream(dec.ctx.h, C.c_void_p(b.data_ptr()), b.numel(), None, None,
                                          C.c_void_p(frames_t.data_ptr()), info["nframes"] + 2,
                                          C.c_void_p(n_t.data_ptr()), dec.opts, C.c_void_p(stream.cuda_stream))
        assert rc == 0, rc

    # Settling: untimed decodes before the W warm-up steps, so that the timed
    # steps see the device's steady state. A burst of 2 GiB decodes runs
    # through a power/clock transient: round 3's (retired) sweep decoder's
    # kernel time rose from ~710 to ~850 us over its first few calls and
    # settled at ~695 us after ~18 (profiles/archive/r03j_c3_dispatch_sequence.json,
    # r03k); the lattice decoder shows none. The timed region is
    # unchanged (exactly K steps), the count is in the JSON line.
    settle = max(0, args.settle - args.warmup)
    for i in range(settle + args.warmup):
        step(i)
    torch.cuda.synchronize()

    # HIP events on the decode stream bracket the timed steps (two events for
    # the whole region, so that no marker sits between the steps): their
    # average is the per-launch time of the decode (k_stream_runs + finish +
    # the launch gaps between steps), the roofline's denominator
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(settle + args.warmup + i)
    ev1.record(stream)
    torch.cuda.synchronize()
    t_own = time.perf_counter() - t0
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = max_over_ranks(dist, torch, t1 - t0, "cpu")
    avg_ms = ev0.elapsed_time(ev1) / args.steps
    decoder = None  # which decoder served the timed steps (the decoder choice, xyws_stream.hip)
    if args.mode == "fused":
        pol = (C.c_uint64 * 5)()
        if dec.ctx.L.xyws_debug_policy(dec.ctx.h, C.c_void_p(stream.cuda_stream), pol) == 0:
            decoder = {0: "runs (k_stream_runs)",
                       2: "runs (k_stream_runs, 512-thread workgroups, 64 KiB segments)",
                       3: "lattice (k_stream_lattice)"}.get(int(pol[4]) & 3)

    if args.stats and rank == 0:  # two extra decodes of copy 0 (keeps its parity)
        names = ["runs", "runs_without_entry", "bad_boundaries", "repairs", "cuts", "spins", "dense_passes",
                 "frames", "scan_segments", "scan_survivors", "scan_undecided", "cyc_scan_filter",
                 "cyc_scan_check", "cyc_scan_resolve", "cyc_dense_entry", "cyc_dense_chase", "cyc_prologue", "cyc_main", "cyc_wait",
                 "cyc_fill", "cyc_chase_sync", "cyc_xor", "cyc_tail", "cyc_prefetch_issue", "cyc_chase_pass",
                 "cyc_pro_fill", "cyc_pro_scan", "cyc_pro_publish", "dense_no_entry", "dense_chase_fail",
                 "dense_mismatch", "dense_overflow", "giveups", "bridges", "steal_requests", "steals",
                 "stolen_segments", "cyc_dense_validate", "cyc_rows", "cyc_serial_chase",
                 "lattice_entries", "cyc_scan_w0", "cyc_scan_bits", "cyc_scan_surv", "s44", "s45", "cyc_stride_pass",
                 "s47"]
        for _ in range(2):
            dec.opts |= _lib.OPT_STATS
            dec.decode(bufs[0], cap=0, count=False, carry=False)
            dec.opts &= ~_lib.OPT_STATS
            out = (C.c_uint64 * _lib.NSTATS)()
            dec.ctx.L.xyws_debug_stats(dec.ctx.h, C.c_void_p(stream.cuda_stream), out)
        st = {k: v for k, v in zip(names, list(out))}
        nrun = max(1, st["runs"] + 1)
        for k in list(st):
            if k.startswith("cyc_"):
                st[k.replace("cyc_", "us_per_run_")] = round(st.pop(k) / nrun / 2100.0, 3)
        print(json.dumps({"stats": st}), flush=True)

    # parity after the timed region: every copy against the reference digest
    # for the parity of its decode count (XOR is an involution)
    if bounds is not None:  # the other ranks' ranges, as often (mod 2) as this one's
        for b, u in zip(bufs, uses):
            for r in range(world):
                if r != rank and u % 2:
                    dec.decode(part(b, r), cap=0, count=False, carry=False)
        torch.cuda.synchronize()
    dev_err = dec.ctx.last_device_error()
    parity = None
    if golden is not None:
        parity = dev_err == 0
        for b, u in zip(bufs, uses):
            parity = parity and device_digest(torch, T, b) == (golden["out_digest"] if u % 2 else golden["in_digest"])
        if n_t is not None and bounds is None:  # the count the frame-table steps returned
            parity = parity and int(n_t.item()) == golden["decoded_frames"]

    per_gpu = args.steps * info["payload_bytes"] / t_own / GIB
    per_gpu_all = [per_gpu]
    if dist:
        per_gpu_all = [None] * world
        dist.all_gather_object(per_gpu_all, round(per_gpu, 3))
    total_payload = info["whole_payload_bytes"] if one else info["payload_bytes"] * world
    value = args.steps * total_payload / elapsed / GIB
    algo_bytes = info["algo_bytes"] + (32 * info["nframes"] if args.frames else 0)  # + the descriptors
    achieved = algo_bytes / (avg_ms * 1e-3) / 1e9
    parity_all = all_ranks(dist, torch, parity, "cpu") if dist else parity

    cpu = None
    host_rate = None
    if rank == 0 and world == 1 and (not args.no_cpu or args.host_path):
        # both legs take the masked input batch: decode copy 0 once more if it is unmasked
        if uses[0] % 2:
            dec.decode(bufs[0], cap=0, count=False, carry=False)
            uses[0] += 1
            torch.cuda.synchronize()
        if not args.no_cpu:
            cpu = cpu_baseline(torch, bufs[0], info, args.cpu_budget)
        if args.host_path and info["nframes"] and args.config != "c4" and golden is not None:
            host_rate = host_path_rate(torch, ws, T, info, bufs[0], golden)
            host_rate["arena"] = arena_path_rate(torch, ws, T, info, bufs[0], golden)

    traffic, traffic_src = pmc_traffic(args.config, args.mode + ("+frames" if args.frames else ""))
    ceiling = None
    if rank == 0 and not args.no_ceiling:
        ceiling = copy_ceiling(torch, ws, bufs[0])
        ceiling["frac_vs_unmask"] = round(achieved / ceiling["unmask_inplace_gbs"], 4)
        ceiling["frac_vs_d2d_copy"] = round(achieved / ceiling["d2d_copy_gbs"], 4)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_calls": settle,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if one else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 masked frames generated in HBM; include/xyws_synth.h)",
            "config": {
                "workload": info["desc"],
                "decoder": decoder,
                "mode": args.mode + " (xyws_decode_stream: boundaries discovered on device)" +
                        (", whole frame table + count returned every step" if args.frames else ""),
                "frames_per_gpu": info["nframes"],
                "batch_bytes_per_gpu": info["size"] if bounds is None else bounds[rank + 1] - bounds[rank],
                "payload_bytes_per_gpu": info["payload_bytes"],
                "batch_copies": ncopies,
                "parallelism": (f"one batch cut at frame boundaries x{world} (xyws_shard_plan_frames), "
                                f"no collective" if one else f"shard-by-frame x{world}, no collective"),
                **({"shard_bounds": bounds} if one else {}),
            },
            "per_gpu_gibs": per_gpu_all,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": algo_bytes,
                "kernel_ms_avg": round(avg_ms, 4),
                "kernel_ms_note": "HIP-event time per decode over the timed steps (the decoder kernel, its "
                                  "in-kernel finish and the gaps between steps); per-kernel: profiles/*_kernel_stats.csv",
                "src_sha": source_hash(),
                "copy_ceiling": ceiling,
            },
            "cpu_baseline": cpu,
            "parity": bool(parity_all) if parity_all is not None else None,
        }
        if host_rate is not None:
            line["host_path"] = host_rate
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
