"""Host-side mirror of xynet's WebSocket frame interface, backed by the gfx950 path.

Names, argument meaning and error behaviour follow the reference headers
(paths relative to the xynet tree):

  websocket_flags                  include/xynet/http/websocket_frame_header.h:42-106
  calc_frame_header_size / _size   :111-131, WS_MAX_FRAME_HEADER_SIZE :134
  websocket_frame_header           :179-224  (xyws_header_build, the reference builder's
                                              bytes; one header, no device work)
  websocket_frame_header_parser    :226-385  (xyws_parser_*: parsed on the device)
  websocket_mask                   include/xynet/http/websocket_frame_mask.h:6-25
  frame_decoder.decode             the batched websocket_recv_data
                                   (example/include/common/websocket.h:110-134)
  encode_frames                    echo_once's replies, batched on the device
                                   (example/websocket/websocket_echo.cpp:18-27)
  classify_frames                  websocket_check_parser_result's policy
                                   (example/include/common/websocket.h:81-108)
  reassemble                       FIN=0 chains -> messages (+ UTF-8 check)
  shard_plan / shard_plan_frames   one batch cut at frame boundaries across devices
                                   (a host-side header walk)

Device buffers are torch uint8 tensors on a ROCm device (PyTorch is used only
for device memory and streams). Every computing call runs HIP kernels from
libxyws.so through its C-ABI; there is no CPU fallback.
"""
import ctypes as C
import enum
import threading

from . import _lib
from ._lib import XYWS_OK, Carry, Frame, XywsError, check

npos = (1 << 64) - 1


class websocket_flags(enum.IntFlag):
    """enum class websocket_flags (websocket_frame_header.h:42-58)."""
    WS_NONE = 0x0
    WS_OP_CONTINUE = 0x0
    WS_OP_TEXT = 0x1
    WS_OP_BINARY = 0x2
    WS_OP_CLOSE = 0x8
    WS_OP_PING = 0x9
    WS_OP_PONG = 0xA
    WS_OP_MASK = 0xF
    WS_FIN = 0x10
    WS_FINAL_FRAME = 0x10
    WS_HAS_MASK = 0x20


def websocket_flags_not_none(flag):
    """websocket_flags_not_none (:61-64)."""
    return bool(int(flag))


def calc_frame_header_size(flags, data_len):
    """detail::calc_frame_header_size (:111-126)."""
    size = 2
    if data_len >= 126:
        size += 8 if data_len > 0xFFFF else 2
    if int(flags) & websocket_flags.WS_HAS_MASK:
        size += 4
    return size


def calc_frame_size(flags, data_len):
    """detail::calc_frame_size (:128-131)."""
    return data_len + calc_frame_header_size(flags, data_len)


WS_MAX_FRAME_HEADER_SIZE = calc_frame_header_size(websocket_flags.WS_HAS_MASK, 0xFFFFFFFF)


def _builder(flags, mask, data_len):
    """detail::websocket_frame_header_builder (:136-175) through xyws_header_build:
    the header bytes; key bytes are written only when `mask` is given (:168-171)."""
    L = _lib.load()
    out = (C.c_uint8 * 16)()
    key = None if mask is None else (C.c_uint8 * 4)(*bytes(mask))
    n = L.xyws_header_build(int(flags) & 0xFF, key, int(data_len) & ((1 << 64) - 1), out)
    return bytes(out[:n])


class websocket_frame_header:
    """class websocket_frame_header (:179-224).

    Reference behaviour is kept in parity mode: the masked constructors store
    the key beside the header and build the header WITHOUT it (:186-188,
    :191-202), so the key bytes on the wire are zero. ``with_key`` builds the
    RFC-correct masked header (client role) instead.
    """

    def __init__(self, flags, data_len, mask=None):
        self._mask = b"\0\0\0\0"
        if mask is not None:
            self._mask = (mask.to_bytes(4, "little") if isinstance(mask, int) else bytes(mask))
        self._header = _builder(flags, None, data_len)

    @classmethod
    def with_key(cls, flags, data_len, key):
        h = cls(flags, data_len)
        key = key.to_bytes(4, "little") if isinstance(key, int) else bytes(key)
        h._mask = key
        h._header = _builder(int(flags) | websocket_flags.WS_HAS_MASK, key, data_len)
        return h

    def view(self):
        return self._header

    def span(self):
        return self._header

    def __len__(self):
        return len(self._header)


# ---------------------------------------------------------------------------
# device plumbing

class Context:
    """An xyws_ctx bound to one HIP device (one per thread and device)."""

    def __init__(self, device=0):
        self.L = _lib.load()
        self.device = device
        h = C.c_void_p()
        check(self.L.xyws_ctx_create(device, C.byref(h)), "xyws_ctx_create")
        self.h = h

    def reserve(self, max_batch_bytes, max_frames=0):
        check(self.L.xyws_ctx_reserve(self.h, max_batch_bytes, max_frames), "xyws_ctx_reserve")

    def reserve_iov(self, max_total_bytes):
        """xyws_ctx_reserve_iov: the buffer-sequence decode's staging buffer."""
        check(self.L.xyws_ctx_reserve_iov(self.h, max_total_bytes), "xyws_ctx_reserve_iov")

    def last_device_error(self):
        """Device error word of the calls since the last read (0 = none);
        synchronizes the device and clears the word (xyws.h)."""
        v = C.c_uint32()
        rc = self.L.xyws_ctx_last_device_error(self.h, C.byref(v))
        if rc not in (XYWS_OK, _lib.XYWS_ERR_DEVICE):
            check(rc, "xyws_ctx_last_device_error")
        return v.value

    def close(self):
        if getattr(self, "h", None):
            self.L.xyws_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


def context(device=None):
    import torch
    dev = torch.cuda.current_device() if device is None else int(device)
    cache = getattr(_tls, "ctx", None)
    if cache is None:
        cache = _tls.ctx = {}
    if dev not in cache:
        cache[dev] = Context(dev)
    return cache[dev]


def _dev_u8(t):
    import torch
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise XywsError(-1, "expected a device-resident torch tensor")
    if t.dtype != torch.uint8 or not t.is_contiguous():
        raise XywsError(-1, "expected a contiguous uint8 tensor")
    return t


def _stream(t):
    import torch
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def websocket_mask(data, mask, i=0):
    """websocket_mask(R&& data, uint32_t mask, size_t i) -> size_t
    (websocket_frame_mask.h:6-25) on a device tensor: in place,
    data[j] ^= bytes(mask)[(i + j) % 4]; returns i + len(data)."""
    t = _dev_u8(data)
    ctx = context(t.device.index)
    key = (C.c_uint8 * 4)(*int(mask & 0xFFFFFFFF).to_bytes(4, "little"))
    out = C.c_uint64()
    check(ctx.L.xyws_unmask(ctx.h, C.c_void_p(t.data_ptr()), t.numel(), key, int(i),
                            C.byref(out), _stream(t)), "xyws_unmask")
    return out.value


def _frames_from_device(frames_t, n):
    import numpy as np
    raw = frames_t[: n * 32].cpu().numpy().tobytes() if n else b""
    arr = (Frame * max(n, 1)).from_buffer_copy(raw.ljust(max(n, 1) * 32, b"\0"))
    return [arr[k] for k in range(n)], np


class DecodeResult:
    """Frames and count of one decode call (device tensors; host copies on demand)."""

    def __init__(self, frames_t, nframes_t, cap):
        self.frames_t = frames_t
        self.nframes_t = nframes_t
        self.cap = cap

    @property
    def nframes(self):
        return int(self.nframes_t.item()) if self.nframes_t is not None else None

    def frames(self):
        if self.frames_t is None:
            return []
        n = min(self.nframes, self.cap)
        return _frames_from_device(self.frames_t, n)[0]


class frame_decoder:
    """Batched, device-resident websocket_recv_data: parse every frame of
    back-to-back batches and unmask payloads in place, carrying a frame or header
    cut by a batch end into the next batch (xyws_decode_stream)."""

    def __init__(self, device=None, serial=False, parse_only=False, small_segments=False, opts=0, ctx=None):
        """serial: the one-lane exact chase (XYWS_OPT_SERIAL_SCAN). small_segments:
        test geometry of the run-parallel decoder (1 KiB runs), so that small
        inputs cross many run boundaries (speculated entries and their repair).
        opts: further XYWS_OPT_* bits. ctx: a Context of its own (default: the
        thread's context for the device)."""
        import torch
        self.ctx = ctx if ctx is not None else context(device)
        self.device = torch.device("cuda", self.ctx.device)
        self.carry_t = torch.zeros(64, dtype=torch.uint8, device=self.device)
        self.opts = (4 if serial else 0) | (1 if parse_only else 0) | (0x200 if small_segments else 0) | opts

    def reset(self):
        self.carry_t.zero_()

    def carry(self):
        return Carry.from_buffer_copy(self.carry_t.cpu().numpy().tobytes())

    def decode(self, buf, cap=0, count=True, carry=True):
        """Decode one batch in place. cap: frame descriptors to return; count:
        return the frame count; carry=False decodes the batch as a fresh stream
        and keeps no state (no carry read or written)."""
        import torch
        t = _dev_u8(buf)
        frames_t = torch.empty(max(cap, 1) * 32, dtype=torch.uint8, device=self.device) if cap else None
        n_t = torch.zeros(1, dtype=torch.int64, device=self.device) if count else None
        cp = C.c_void_p(self.carry_t.data_ptr()) if carry else None
        check(self.ctx.L.xyws_decode_stream(
            self.ctx.h, C.c_void_p(t.data_ptr()), t.numel(), cp, cp,
            C.c_void_p(frames_t.data_ptr()) if frames_t is not None else None, cap,
            C.c_void_p(n_t.data_ptr()) if n_t is not None else None, self.opts, _stream(t)),
            "xyws_decode_stream")
        return DecodeResult(frames_t, n_t, cap)

    def decode_iov(self, bufs, cap=0, count=True, carry=True):
        """Decode a buffer sequence (device uint8 tensors, one recv's pieces)
        as ONE stream, every piece in place (xyws_decode_stream_iov: three
        launches whatever the piece count). Descriptor offsets count bytes
        across the pieces in order."""
        import torch
        ts = [_dev_u8(b) for b in bufs]
        arr = (C.c_uint64 * (2 * max(len(ts), 1)))()
        for k, t in enumerate(ts):
            arr[2 * k], arr[2 * k + 1] = t.data_ptr(), t.numel()
        frames_t = torch.empty(max(cap, 1) * 32, dtype=torch.uint8, device=self.device) if cap else None
        n_t = torch.zeros(1, dtype=torch.int64, device=self.device) if count else None
        cp = C.c_void_p(self.carry_t.data_ptr()) if carry else None
        check(self.ctx.L.xyws_decode_stream_iov(
            self.ctx.h, C.cast(arr, C.c_void_p), len(ts), cp, cp,
            C.c_void_p(frames_t.data_ptr()) if frames_t is not None else None, cap,
            C.c_void_p(n_t.data_ptr()) if n_t is not None else None, self.opts,
            _stream(ts[0]) if ts else C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
            "xyws_decode_stream_iov")
        return DecodeResult(frames_t, n_t, cap)


def decode_indexed(buf, starts, frames=True, parse_only=False):
    """Frames at known offsets (ascending): parse + unmask in place."""
    import torch
    t = _dev_u8(buf)
    ctx = context(t.device.index)
    st = torch.as_tensor(starts, dtype=torch.int64).to(t.device)
    n = st.numel()
    frames_t = torch.empty(max(n, 1) * 32, dtype=torch.uint8, device=t.device) if frames else None
    check(ctx.L.xyws_decode_indexed(
        ctx.h, C.c_void_p(t.data_ptr()), t.numel(), C.c_void_p(st.data_ptr()), n,
        C.c_void_p(frames_t.data_ptr()) if frames_t is not None else None,
        1 if parse_only else 0, _stream(t)), "xyws_decode_indexed")
    res = DecodeResult(frames_t, None, n)
    res.nframes_t = torch.tensor([n], dtype=torch.int64)
    return res


class websocket_frame_header_parser:
    """websocket_frame_header_parser (:226-385) through xyws_parser_* (C-ABI).

    parse(data) takes bytes (host) or a device uint8 tensor and returns the
    number of bytes consumed in THIS call up to the end of the header, or
    ``npos`` while the header is incomplete; once a header completed, further
    input returns npos until reset() (:378-384). result() returns (flags,
    mask_uint32_t, length) (websocket.h:121-128). The bytes are parsed on the
    device (stream decoder, parse-only, device-resident carry).
    """
    npos = npos

    def __init__(self, device=None):
        import torch
        self.ctx = context(device)
        self.L = self.ctx.L
        h = C.c_void_p()
        check(self.L.xyws_parser_create(self.ctx.h, C.byref(h)), "xyws_parser_create")
        self.h = h
        self._stream = C.c_void_p(torch.cuda.current_stream(self.ctx.device).cuda_stream)

    def __del__(self):
        try:
            if self.h:
                self.L.xyws_parser_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def reset(self):
        check(self.L.xyws_parser_reset(self.h), "xyws_parser_reset")

    def parse(self, data):
        import torch
        consumed = C.c_uint64()
        if isinstance(data, torch.Tensor):
            t = _dev_u8(data)
            ptr, n = C.c_void_p(t.data_ptr()), t.numel()
            check(self.L.xyws_parser_parse(self.h, ptr, n, C.byref(consumed), _stream(t)), "xyws_parser_parse")
        else:
            b = bytes(data)
            buf = C.create_string_buffer(b, max(len(b), 1))
            check(self.L.xyws_parser_parse(self.h, buf, len(b), C.byref(consumed), self._stream),
                  "xyws_parser_parse")
        return consumed.value

    def _res(self):
        f, ln = C.c_uint8(), C.c_uint64()
        key = (C.c_uint8 * 4)()
        check(self.L.xyws_parser_result(self.h, C.byref(f), key, C.byref(ln)), "xyws_parser_result")
        return websocket_flags(f.value), int.from_bytes(bytes(key), "little"), ln.value

    def flags(self):
        return self._res()[0]

    def length(self):
        return self._res()[2]

    def mask_uint32_t(self):
        return self._res()[1]

    def mask(self):
        return self._res()[1].to_bytes(4, "little")

    def result(self):
        return self._res()


# ---------------------------------------------------------------------------
# the callers either side of the decode path (xyws_frames.hip)

def _opt_ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def encode_frames(src, frames_t, n, flags, dev_n=None, enc_opts=0, keys=None, verdicts=None,
                  action_mask=0, out=None, offsets=None):
    """echo_once's replies for a decoded frame table, on the device
    (xyws_encode_frames). src: the decoded batch (device uint8); frames_t:
    n xyws_frame records (device uint8, n*32 bytes); keys: device uint8 (4 per
    frame) for client-role masking. Returns (out, out_len tensor)."""
    import torch
    t = _dev_u8(src)
    ctx = context(t.device.index)
    olen = torch.zeros(1, dtype=torch.int64, device=t.device)
    if out is None:
        raise XywsError(-1, "encode_frames needs an output tensor (size it with encode_size)")
    check(ctx.L.xyws_encode_frames(ctx.h, C.c_void_p(t.data_ptr()), t.numel(), _opt_ptr(frames_t), n,
                                   _opt_ptr(dev_n), int(flags) & 0xFF, enc_opts, _opt_ptr(keys),
                                   _opt_ptr(verdicts), action_mask, C.c_void_p(out.data_ptr()), out.numel(),
                                   _opt_ptr(offsets), C.c_void_p(olen.data_ptr()), _stream(t)),
          "xyws_encode_frames")
    return out, olen


def classify_frames(src, frames_t, n, max_payload, policy=0, dev_n=None):
    """websocket_check_parser_result per frame (xyws_classify_frames): returns
    (verdicts tensor (n*8 bytes), first-close tensor)."""
    import torch
    t = _dev_u8(src)
    ctx = context(t.device.index)
    verd = torch.zeros(max(n, 1) * 8, dtype=torch.uint8, device=t.device)
    first = torch.zeros(1, dtype=torch.int64, device=t.device)
    check(ctx.L.xyws_classify_frames(ctx.h, C.c_void_p(t.data_ptr()), t.numel(), _opt_ptr(frames_t), n,
                                     _opt_ptr(dev_n), max_payload, policy, C.c_void_p(verd.data_ptr()),
                                     C.c_void_p(first.data_ptr()), _stream(t)), "xyws_classify_frames")
    return verd, first


def reassemble(src, frames_t, n, opts=0, out_cap=None, msg_cap=None, dev_n=None):
    """FIN=0 chains gathered into messages (xyws_reassemble): returns (out,
    messages tensor (msg_cap*40 bytes), count tensor)."""
    import torch
    t = _dev_u8(src)
    ctx = context(t.device.index)
    cap = t.numel() if out_cap is None else out_cap
    mcap = max(n, 1) if msg_cap is None else msg_cap
    out = torch.zeros(max(cap, 1), dtype=torch.uint8, device=t.device)
    msgs = torch.zeros(max(mcap, 1) * 40, dtype=torch.uint8, device=t.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=t.device)
    check(ctx.L.xyws_reassemble(ctx.h, C.c_void_p(t.data_ptr()), t.numel(), _opt_ptr(frames_t), n, _opt_ptr(dev_n),
                                opts, C.c_void_p(out.data_ptr()), cap, C.c_void_p(msgs.data_ptr()), mcap,
                                C.c_void_p(cnt.data_ptr()), _stream(t)), "xyws_reassemble")
    return out, msgs, cnt


class RecvArena:
    """A connection's receive arena (xyws_arena_*): recv into pinned host
    memory, decode on the device with the connection's carry, results and the
    unmasked bytes back in place; each completion writes 1 to `eventfd` (the
    fd an io_uring loop keeps a poll_add on, io_service.h:362-381)."""

    def __init__(self, nbytes, max_frames, eventfd=-1, device=None, host=None):
        self.ctx = context(device)
        self.L = self.ctx.L
        h = C.c_void_p()
        check(self.L.xyws_arena_create(self.ctx.h, host, nbytes, max_frames, eventfd, C.byref(h)),
              "xyws_arena_create")
        self.h = h
        self.nbytes = nbytes
        self.max_frames = max_frames
        self.host_ptr = self.L.xyws_arena_host(h)

    def view(self):
        """The receive area as a writable memoryview (pinned host memory)."""
        return (C.c_uint8 * self.nbytes).from_address(self.host_ptr)

    def submit(self, offset, length, opts=0):
        seq = C.c_uint64()
        rc = self.L.xyws_arena_submit(self.h, offset, length, opts, C.byref(seq))
        if rc == _lib.XYWS_ERR_AGAIN:
            return None
        check(rc, "xyws_arena_submit")
        return seq.value

    def poll(self, seq):
        res = _lib.ArenaResult()
        rc = self.L.xyws_arena_poll(self.h, seq, C.byref(res))
        if rc == _lib.XYWS_ERR_AGAIN:
            return None
        check(rc, "xyws_arena_poll")
        return res

    def wait(self, seq):
        res = _lib.ArenaResult()
        check(self.L.xyws_arena_wait(self.h, seq, C.byref(res)), "xyws_arena_wait")
        return res

    @staticmethod
    def frames_of(res, max_frames):
        return [res.frames[i] for i in range(min(res.nframes, max_frames))]

    def close(self):
        if getattr(self, "h", None):
            self.L.xyws_arena_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_plan(batch, n_shards, carry=None):
    """Cut one batch of back-to-back frames (host bytes: bytes, bytearray,
    numpy uint8 array, or a CPU uint8 tensor) into n_shards byte ranges at
    frame boundaries, balanced by bytes (xyws_shard_plan). Returns the
    n_shards + 1 bounds; shard k is batch[bounds[k]:bounds[k+1]], shard 0
    continues from `carry` (a Carry or None), the others start fresh."""
    import numpy as np
    L = _lib.load()
    if hasattr(batch, "numpy"):
        batch = batch.numpy()
    arr = np.ascontiguousarray(np.frombuffer(batch, dtype=np.uint8) if isinstance(batch, (bytes, bytearray))
                               else batch, dtype=np.uint8)
    out = (C.c_uint64 * (n_shards + 1))()
    cin = C.byref(carry) if carry is not None else None
    check(L.xyws_shard_plan(C.c_void_p(arr.ctypes.data) if arr.size else None, arr.size, cin, int(n_shards), out),
          "xyws_shard_plan")
    return list(out)


def shard_plan_frames(frames, length, n_shards):
    """shard_plan from a host frame table (a sequence of Frame, or a ctypes
    Frame array), frame_off ascending (xyws_shard_plan_frames)."""
    L = _lib.load()
    n = len(frames)
    arr = frames if isinstance(frames, C.Array) else \
        (Frame * max(n, 1)).from_buffer_copy(b"".join(bytes(f) for f in frames).ljust(32 * max(n, 1), b"\0"))
    out = (C.c_uint64 * (n_shards + 1))()
    check(L.xyws_shard_plan_frames(arr, n, int(length), int(n_shards), out), "xyws_shard_plan_frames")
    return list(out)
