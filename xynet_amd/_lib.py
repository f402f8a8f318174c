"""ctypes binding of libxyws.so (include/xyws.h) and libxyws_tools.so.

The decode path has no CPU fallback: if the in-tree HIP library is missing or a
device is absent, calls raise XywsError instead of computing anything on the
host.
"""
import ctypes as C
import os
import re

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
HEADER = os.path.join(ROOT, "include", "xyws.h")

XYWS_OK = 0
XYWS_ERR_DEVICE = -5
NSTATS = 48  # XYWS_NSTATS (xyws_stream.h)
R_WORDS = 32  # u64 words per run record (xyws_stream.hip)
# internal decode options (xyws_stream.h; not part of include/xyws.h)
OPT_STATS = 0x100
OPT_SMALL_SEG = 0x200
OPT_WG512 = 0x40000
OPT_NO_LATENTRY = 0x4000   # run decoder experiment: no lattice entry
OPT_WG1024 = 0x8000        # the run decoder's default geometry, whatever the geometry choice would take
OPT_TEST_GIVEUP = 0x100000
OPT_STEAL = 0x400000
OPT_TEST_STEAL = 0x800000
OPT_RUNS = 0x80000000      # the run decoder whatever the decoder choice would take
OPT_LATTICE = 0x400        # the lattice decoder first (the run decoder after it takes what it leaves)
OPT_NO_LATDEC = 0x800      # never the lattice decoder
OPT_BIGSCAN = 0x4000000    # tests: the entry scans' one-pass filter whatever the previous call found
OPT_NO_BIGSCAN = 0x40000000  # the entry scans' window-0 pass whatever the previous call found
OPT_TEST_LATSPEC = 0x10    # tests (lattice decoder): every store speculative (undone at the end of the work)
OPT_TEST_LATDUMP = 0x20    # tests (lattice decoder): every speculative-store list undone by the finisher
# debug stats indices (xyws_stream.hip)
ST_RUNS, ST_NONE, ST_BAD, ST_REPAIR, ST_CUT, ST_SPIN, ST_SEGS, ST_FRAMES = range(8)
ST_GIVEUP, ST_BRIDGE, ST_STEAL_REQ, ST_STEAL_ACC, ST_STEAL_SEGS = 32, 33, 34, 35, 36
ST_P_LATTICE = 40  # run decoder: runs whose entry the lattice gave (find_entry)
ERRORS = {-1: "invalid argument", -2: "HIP runtime error", -3: "device allocation failed",
          -4: "scratch capacity exceeded", -5: "device-side error", -6: "not complete yet"}


class XywsError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"xyws error {code} ({ERRORS.get(code, '?')}){': ' + what if what else ''}")


class Frame(C.Structure):
    """xyws_frame (include/xyws.h), 32 bytes."""
    _fields_ = [("frame_off", C.c_int64), ("payload_off", C.c_int64),
                ("payload_len", C.c_uint64), ("key", C.c_uint8 * 4),
                ("flags", C.c_uint8), ("hdr_len", C.c_uint8),
                ("status", C.c_uint8), ("reserved", C.c_uint8)]


class Carry(C.Structure):
    """xyws_carry (include/xyws.h), 64 bytes."""
    _fields_ = [("payload_remaining", C.c_uint64), ("phase", C.c_uint64),
                ("frames_total", C.c_uint64), ("key", C.c_uint8 * 4),
                ("hdr_len", C.c_uint8), ("hdr", C.c_uint8 * 14),
                ("reserved", C.c_uint8 * 21)]


class Verdict(C.Structure):
    """xyws_verdict (include/xyws.h), 8 bytes."""
    _fields_ = [("close_code", C.c_uint16), ("peer_code", C.c_uint16), ("action", C.c_uint8),
                ("reserved", C.c_uint8 * 3)]


class Message(C.Structure):
    """xyws_message (include/xyws.h), 40 bytes."""
    _fields_ = [("first_frame", C.c_uint64), ("nframes", C.c_uint64), ("out_off", C.c_uint64),
                ("length", C.c_uint64), ("status", C.c_uint32), ("opcode", C.c_uint8),
                ("reserved", C.c_uint8 * 3)]


class ArenaResult(C.Structure):
    """xyws_arena_result (include/xyws.h)."""
    _fields_ = [("seq", C.c_uint64), ("offset", C.c_uint64), ("len", C.c_uint64), ("nframes", C.c_uint64),
                ("frames", C.POINTER(Frame)), ("carry", Carry)]


assert C.sizeof(Frame) == 32 and C.sizeof(Carry) == 64
assert C.sizeof(ArenaResult) == 104
XYWS_ERR_AGAIN = -6
ARENA_SLOTS = 8
assert C.sizeof(Verdict) == 8 and C.sizeof(Message) == 40
NPOS = (1 << 64) - 1
ENC_FRAME_OPCODE = 0x1
ACT_DATA, ACT_PING, ACT_PONG, ACT_CLOSE = 0, 1, 2, 3
POL_FRAGMENTS, POL_UNMASKED, POL_STRICT = 0x1, 0x2, 0x4
REASM_UTF8 = 0x1
MSG_COMPLETE, MSG_UTF8_BAD, MSG_INTERRUPTED, MSG_TRUNCATED, MSG_ORPHANS = 0x1, 0x2, 0x4, 0x8, 0x10

_lib = None
_tools = None


def declared_symbols(header=HEADER):
    """Function names declared in include/xyws.h."""
    src = open(header).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*|uint64_t|void\s*\*|void)\s*(xyws_\w+)\s*\(",
                                 src, re.M)))


def lib_path(name="libxyws.so"):
    return os.path.join(PKG, name)


def load():
    """Load libxyws.so (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    # XYWS_LIB: an alternative in-tree build of the same library (A/B timing
    # of compile-time variants; scripts/exp_variants.sh)
    path = os.environ.get("XYWS_LIB") or lib_path()
    if not os.path.exists(path):
        raise XywsError(-2, f"{path} missing: build it with `python -m xynet_amd.build`")
    L = C.CDLL(path)
    u64, u32, u8, vp, i32 = C.c_uint64, C.c_uint32, C.c_uint8, C.c_void_p, C.c_int
    L.xyws_abi_version.restype = i32
    L.xyws_strerror.restype = C.c_char_p
    L.xyws_strerror.argtypes = [i32]
    L.xyws_ctx_create.restype = i32
    L.xyws_ctx_create.argtypes = [i32, C.POINTER(vp)]
    L.xyws_ctx_destroy.restype = i32
    L.xyws_ctx_destroy.argtypes = [vp]
    L.xyws_ctx_reserve.restype = i32
    L.xyws_ctx_reserve.argtypes = [vp, u64, u64]
    L.xyws_ctx_reserve_iov.restype = i32
    L.xyws_ctx_reserve_iov.argtypes = [vp, u64]
    L.xyws_ctx_last_device_error.restype = i32
    L.xyws_ctx_last_device_error.argtypes = [vp, C.POINTER(u32)]
    L.xyws_unmask.restype = i32
    L.xyws_unmask.argtypes = [vp, vp, u64, vp, u64, C.POINTER(u64), vp]
    L.xyws_mask_bytes.restype = i32
    L.xyws_mask_bytes.argtypes = [vp, vp, u64, vp, u64, C.POINTER(u64), vp]
    L.xyws_decode_indexed.restype = i32
    L.xyws_decode_indexed.argtypes = [vp, vp, u64, vp, u64, vp, u32, vp]
    L.xyws_debug_stats.restype = i32
    L.xyws_debug_stats.argtypes = [vp, vp, C.POINTER(C.c_uint64)]
    L.xyws_debug_policy.restype = i32
    L.xyws_debug_policy.argtypes = [vp, vp, C.POINTER(C.c_uint64)]
    L.xyws_debug_lattice.restype = i32
    L.xyws_debug_lattice.argtypes = [vp, vp, C.POINTER(C.c_uint64)]
    L.xyws_debug_records.restype = C.c_int64
    L.xyws_debug_records.argtypes = [vp, vp, C.POINTER(C.c_uint64), u64]
    L.xyws_decode_stream.restype = i32
    L.xyws_decode_stream.argtypes = [vp, vp, u64, vp, vp, vp, u64, vp, u32, vp]
    L.xyws_decode_stream_iov.restype = i32
    L.xyws_decode_stream_iov.argtypes = [vp, vp, u32, vp, vp, vp, u64, vp, u32, vp]
    # ABI 2
    L.xyws_parser_create.restype = i32
    L.xyws_parser_create.argtypes = [vp, C.POINTER(vp)]
    L.xyws_parser_destroy.restype = i32
    L.xyws_parser_destroy.argtypes = [vp]
    L.xyws_parser_reset.restype = i32
    L.xyws_parser_reset.argtypes = [vp]
    L.xyws_parser_parse.restype = i32
    L.xyws_parser_parse.argtypes = [vp, vp, u64, C.POINTER(u64), vp]
    L.xyws_parser_result.restype = i32
    L.xyws_parser_result.argtypes = [vp, C.POINTER(u8), vp, C.POINTER(u64)]
    L.xyws_header_build.restype = u64
    L.xyws_header_build.argtypes = [u8, vp, u64, vp]
    L.xyws_encode_frames.restype = i32
    L.xyws_encode_frames.argtypes = [vp, vp, u64, vp, u64, vp, u8, u32, vp, vp, u32, vp, u64, vp, vp, vp]
    L.xyws_classify_frames.restype = i32
    L.xyws_classify_frames.argtypes = [vp, vp, u64, vp, u64, vp, u64, u32, vp, vp, vp]
    L.xyws_reassemble.restype = i32
    L.xyws_reassemble.argtypes = [vp, vp, u64, vp, u64, vp, u32, vp, u64, vp, u64, vp, vp]
    L.xyws_arena_create.restype = i32
    L.xyws_arena_create.argtypes = [vp, vp, u64, u64, i32, C.POINTER(vp)]
    L.xyws_arena_destroy.restype = i32
    L.xyws_arena_destroy.argtypes = [vp]
    L.xyws_arena_host.restype = vp
    L.xyws_arena_host.argtypes = [vp]
    L.xyws_arena_submit.restype = i32
    L.xyws_arena_submit.argtypes = [vp, u64, u64, u32, C.POINTER(u64)]
    L.xyws_arena_poll.restype = i32
    L.xyws_arena_poll.argtypes = [vp, u64, vp]
    L.xyws_arena_wait.restype = i32
    L.xyws_arena_wait.argtypes = [vp, u64, vp]
    L.xyws_notifier_create.restype = i32
    L.xyws_notifier_create.argtypes = [i32, C.POINTER(vp)]
    L.xyws_notifier_destroy.restype = i32
    L.xyws_notifier_destroy.argtypes = [vp]
    L.xyws_notifier_signal.restype = i32
    L.xyws_notifier_signal.argtypes = [vp, u64]
    L.xyws_notifier_completed.restype = u64
    L.xyws_notifier_completed.argtypes = [vp]
    L.xyws_shard_plan.restype = i32
    L.xyws_shard_plan.argtypes = [vp, u64, vp, u32, C.POINTER(u64)]
    L.xyws_shard_plan_frames.restype = i32
    L.xyws_shard_plan_frames.argtypes = [vp, u64, u64, u32, C.POINTER(u64)]
    _lib = L
    return L


def load_tools():
    global _tools
    if _tools is not None:
        return _tools
    path = lib_path("libxyws_tools.so")
    if not os.path.exists(path):
        raise XywsError(-2, f"{path} missing: build it with `python -m xynet_amd.build`")
    T = C.CDLL(path)
    u64, u8, vp, i32 = C.c_uint64, C.c_uint8, C.c_void_p, C.c_int
    T.xyws_tools_fill_uniform.restype = i32
    T.xyws_tools_fill_uniform.argtypes = [vp, u64, u64, u8, u64, vp]
    T.xyws_tools_mixed_table.restype = u64
    T.xyws_tools_mixed_table.argtypes = [u64, u64, vp, u64, C.POINTER(u64)]
    T.xyws_tools_fill_mixed.restype = i32
    T.xyws_tools_fill_mixed.argtypes = [vp, u64, vp, u64, u64, vp]
    T.xyws_tools_digest.restype = i32
    T.xyws_tools_digest.argtypes = [vp, u64, vp, vp, vp]
    _tools = T
    return T


def check(rc, what=""):
    if rc != XYWS_OK:
        raise XywsError(rc, what)
    return rc
