"""The io_uring side of the boundary (include/xyws.h, recv arenas; reference
anchors include/xynet/socket/impl/recv_all.h:86-121 and
include/xynet/io_service.h:362-381).

- CPU: the completion notifier alone: a foreign thread marks submissions
  complete and writes the eventfd; the loop waits on the fd with poll() (as
  the ring does with poll_add) and reads the completed sequence.
- GPU: a stream received in recv-sized pieces (cut anywhere, 1-byte pieces
  included) into a pinned arena, decoded piece by piece with the carry chained
  on the device, completions taken from the eventfd: the bytes unmasked in
  place and the frame list equal the oracle's decode of the unsplit stream.
"""
import ctypes as C
import os
import select
import threading
import time

import numpy as np
import pytest

import streams

torch = pytest.importorskip("torch")


def test_notifier_eventfd_handshake():
    from xynet_amd import _lib
    L = _lib.load()
    fd = os.eventfd(0, os.EFD_NONBLOCK)
    h = C.c_void_p()
    assert L.xyws_notifier_create(fd, C.byref(h)) == 0
    try:
        def producer():
            for seq in range(5):
                time.sleep(0.01)
                assert L.xyws_notifier_signal(h, seq) == 0

        th = threading.Thread(target=producer)
        th.start()
        p = select.poll()
        p.register(fd, select.POLLIN)
        got = 0
        deadline = time.time() + 10
        while L.xyws_notifier_completed(h) < 5 and time.time() < deadline:
            if p.poll(1000):
                got += os.eventfd_read(fd)
        th.join()
        try:
            got += os.eventfd_read(fd)
        except BlockingIOError:
            pass
        assert L.xyws_notifier_completed(h) == 5
        assert got == 5
        # completion is in order: an older sequence number never lowers it
        L.xyws_notifier_signal(h, 2)
        assert L.xyws_notifier_completed(h) == 5
    finally:
        L.xyws_notifier_destroy(h)
        os.close(fd)


def _pieces(rng, n, count):
    cuts = sorted(set(rng.below(n + 1) for _ in range(count)) | {0, n})
    out = [(a, b - a) for a, b in zip(cuts, cuts[1:])]
    # a few 1-byte pieces (a header trickling in byte by byte)
    return out


def _abs_frames(res, max_frames):
    out = []
    for i in range(min(res.nframes, max_frames)):
        f = res.frames[i]
        out.append((f.frame_off + res.offset, f.payload_off + res.offset, f.payload_len, bytes(f.key), f.flags,
                    f.hdr_len, f.status & ~1))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("case,pieces,registered", [
    ("random_frames_200", 40, False), ("fragments", 25, False), ("lengths", 60, True),
    ("tiny_frames", 300, False), ("trunc_payload", 7, False)])
def test_arena_round_trip_in_recv_pieces(oracle, case, pieces, registered):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from xynet_amd import websocket as ws
    wire = streams.case_bytes(case)
    n = len(wire)
    rng = streams.SplitMix(n + pieces)
    parts = _pieces(rng, n, pieces)
    parts += [(n, 0)]  # an empty recv (peer idle) is a valid submission
    fd = os.eventfd(0, os.EFD_NONBLOCK)
    host = (C.c_uint8 * n).from_buffer_copy(wire) if registered else None
    max_frames = n // 2 + 2
    arena = ws.RecvArena(n, max_frames, eventfd=fd, host=C.addressof(host) if registered else None)
    try:
        if not registered:
            C.memmove(arena.host_ptr, wire, n)
        p = select.poll()
        p.register(fd, select.POLLIN)
        seqs, results, pending = [], {}, []
        for off, ln in parts:
            while True:
                s = arena.submit(off, ln)
                if s is not None:
                    break
                p.poll(1000)  # every slot in flight: wait for a completion
                os.eventfd_read(fd)
                for q in list(pending):
                    r = arena.poll(q)
                    if r is not None:
                        results[q] = _abs_frames(r, max_frames)
                        pending.remove(q)
            seqs.append(s)
            pending.append(s)
        deadline = time.time() + 30
        while pending and time.time() < deadline:
            if p.poll(1000):
                os.eventfd_read(fd)
            for q in list(pending):
                r = arena.poll(q)
                if r is not None:
                    results[q] = _abs_frames(r, max_frames)
                    last = r
                    pending.remove(q)
        assert not pending, "completions never arrived on the eventfd"
        got = bytes(C.string_at(arena.host_ptr, n))
        ref = np.frombuffer(wire, np.uint8).copy()
        ofr, oc, on = oracle.decode_stream(ref)
        assert got == ref.tobytes()
        frames = [f for s in seqs for f in results[s]]
        want = [(f.frame_off, f.payload_off, f.payload_len, bytes(f.key), f.flags, f.hdr_len, f.status & ~1)
                for f in ofr]
        assert frames == want
        assert (last.carry.payload_remaining, last.carry.phase, last.carry.frames_total,
                bytes(last.carry.key), last.carry.hdr_len) == (oc.payload_remaining, oc.phase, oc.frames_total,
                                                               bytes(oc.key), oc.hdr_len)
        assert ws.context().last_device_error() == 0
    finally:
        arena.close()
        os.close(fd)
