"""ctypes bindings for the CPU checkers (TEST INFRASTRUCTURE ONLY).

- ``Oracle``: oracle/liboracle.so, the C restatement of the reference hot path
  (oracle/xyws_oracle.c; cites include/xynet/http/websocket_frame_header.h and
  websocket_frame_mask.h line by line).
- ``Reference``: oracle/_ref/libxynet_ref.so, the reference's own headers behind
  a C-ABI harness (oracle/ref_harness.cpp), built in the survey container only.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
NPOS = (1 << 64) - 1


class Frame(C.Structure):
    """Mirror of xyws_frame (include/xyws.h)."""
    _fields_ = [("frame_off", C.c_int64), ("payload_off", C.c_int64),
                ("payload_len", C.c_uint64), ("key", C.c_uint8 * 4),
                ("flags", C.c_uint8), ("hdr_len", C.c_uint8),
                ("status", C.c_uint8), ("reserved", C.c_uint8)]

    def as_tuple(self, with_status=True):
        t = (self.frame_off, self.payload_off, self.payload_len, bytes(self.key),
             self.flags, self.hdr_len)
        return t + (self.status,) if with_status else t


class Carry(C.Structure):
    """Mirror of xyws_carry (include/xyws.h)."""
    _fields_ = [("payload_remaining", C.c_uint64), ("phase", C.c_uint64),
                ("frames_total", C.c_uint64), ("key", C.c_uint8 * 4),
                ("hdr_len", C.c_uint8), ("hdr", C.c_uint8 * 14),
                ("reserved", C.c_uint8 * 21)]

    def as_tuple(self):
        return (self.payload_remaining, self.phase, self.frames_total, bytes(self.key),
                self.hdr_len, bytes(self.hdr[: self.hdr_len]))


assert C.sizeof(Frame) == 32 and C.sizeof(Carry) == 64


class Verdict(C.Structure):
    """Mirror of xyws_verdict (include/xyws.h)."""
    _fields_ = [("close_code", C.c_uint16), ("peer_code", C.c_uint16), ("action", C.c_uint8),
                ("reserved", C.c_uint8 * 3)]

    def as_tuple(self):
        return (self.close_code, self.peer_code, self.action)


class Message(C.Structure):
    """Mirror of xyws_message (include/xyws.h)."""
    _fields_ = [("first_frame", C.c_uint64), ("nframes", C.c_uint64), ("out_off", C.c_uint64),
                ("length", C.c_uint64), ("status", C.c_uint32), ("opcode", C.c_uint8),
                ("reserved", C.c_uint8 * 3)]

    def as_tuple(self):
        return (self.first_frame, self.nframes, self.out_off, self.length, self.status, self.opcode)


assert C.sizeof(Verdict) == 8 and C.sizeof(Message) == 40


class SynthFrame(C.Structure):
    """Mirror of xyws_synth_frame (include/xyws_synth.h)."""
    _fields_ = [("off", C.c_uint64), ("plen", C.c_uint64), ("draw", C.c_uint64),
                ("b0", C.c_uint8), ("hlen", C.c_uint8), ("pad", C.c_uint8 * 6)]


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def build(quiet=True):
    """Compile liboracle.so (and oracle/_ref when the reference tree exists)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


def oracle_lib_path(opt="O2"):
    return os.path.join(HERE, "liboracle.so" if opt == "O2" else "liboracle_O0.so")


class Oracle:
    def __init__(self, path=None):
        path = path or oracle_lib_path("O2")
        if not os.path.exists(path):
            build()
        L = self.L = C.CDLL(path)
        u64, u32, u8, vp = C.c_uint64, C.c_uint32, C.c_uint8, C.c_void_p
        L.oracle_parser_parse.restype = u64
        L.oracle_parser_parse.argtypes = [vp, vp, u64]
        L.oracle_parser_reset.argtypes = [vp]
        L.oracle_parser_mask_u32.restype = u32
        L.oracle_parser_mask_u32.argtypes = [vp]
        L.oracle_parser_flags.restype = u8
        L.oracle_parser_flags.argtypes = [vp]
        L.oracle_parser_length.restype = u64
        L.oracle_parser_length.argtypes = [vp]
        L.oracle_mask.restype = u64
        L.oracle_mask.argtypes = [vp, u64, u32, u64]
        L.oracle_calc_frame_header_size.restype = u64
        L.oracle_calc_frame_header_size.argtypes = [u8, u64]
        L.oracle_header_build.restype = u64
        L.oracle_header_build.argtypes = [vp, u8, vp, u64]
        L.oracle_decode_stream.restype = u64
        L.oracle_decode_stream.argtypes = [vp, u64, vp, vp, vp, u64]
        L.oracle_decode_indexed.argtypes = [vp, u64, vp, u64, vp]
        L.oracle_digest.restype = u64
        L.oracle_digest.argtypes = [vp, u64]
        L.oracle_fill_uniform.argtypes = [vp, u64, u64, u8, u64]
        L.oracle_mixed_table.restype = u64
        L.oracle_mixed_table.argtypes = [u64, u64, vp, u64, C.POINTER(u64)]
        L.oracle_fill_mixed.argtypes = [vp, vp, u64, u64]
        L.oracle_decode_batch_mt.restype = u64
        L.oracle_decode_batch_mt.argtypes = [vp, u64, C.c_int]
        L.oracle_encode_frames.restype = u64
        L.oracle_encode_frames.argtypes = [vp, u64, vp, u64, u8, u32, vp, vp, u32, vp, u64, vp]
        L.oracle_classify.argtypes = [vp, u64, vp, u64, u64, u32, vp, C.POINTER(u64)]
        L.oracle_utf8_valid.restype = C.c_int
        L.oracle_utf8_valid.argtypes = [vp, u64, C.c_int]
        L.oracle_reassemble.restype = u64
        L.oracle_reassemble.argtypes = [vp, u64, vp, u64, u32, vp, u64, vp, u64]

    # --- parser object (websocket_frame_header_parser) ---
    class Parser:
        def __init__(self, L):
            self.L = L
            self.buf = C.create_string_buffer(40)
            L.oracle_parser_reset(self.buf)

        def parse(self, data: bytes):
            b = C.create_string_buffer(bytes(data), max(len(data), 1))
            return self.L.oracle_parser_parse(self.buf, b, len(data))

        def reset(self):
            self.L.oracle_parser_reset(self.buf)

        def result(self):
            return (self.L.oracle_parser_flags(self.buf), self.L.oracle_parser_mask_u32(self.buf),
                    self.L.oracle_parser_length(self.buf))

    def parser(self):
        return Oracle.Parser(self.L)

    def mask(self, arr: np.ndarray, key_u32: int, phase: int) -> int:
        return self.L.oracle_mask(_ptr(arr), arr.size, key_u32, phase)

    def header_build(self, flags, mask, length):
        out = np.zeros(16, np.uint8)
        mk = None if mask is None else np.frombuffer(bytes(mask), np.uint8).copy()
        n = self.L.oracle_header_build(_ptr(out), flags, _ptr(mk), length)
        return out[:n].tobytes()

    def calc_frame_header_size(self, flags, length):
        return self.L.oracle_calc_frame_header_size(flags, length)

    def decode_stream(self, buf: np.ndarray, carry_in=None, cap=None):
        """In place. Returns (frames list, carry_out, nframes)."""
        n_est = cap if cap is not None else max(16, buf.size // 2 + 2)
        frames = (Frame * n_est)()
        cout = Carry()
        n = self.L.oracle_decode_stream(_ptr(buf), buf.size,
                                        C.byref(carry_in) if carry_in is not None else None,
                                        C.byref(cout), frames, n_est)
        return [frames[i] for i in range(min(n, n_est))], cout, n

    def decode_stream_raw(self, buf: np.ndarray, cap, carry_in=None):
        """decode_stream with the descriptors as one uint8 array (cap * 32 B)."""
        raw = np.zeros(max(cap, 1) * 32, np.uint8)
        cout = Carry()
        n = self.L.oracle_decode_stream(_ptr(buf), buf.size,
                                        C.byref(carry_in) if carry_in is not None else None,
                                        C.byref(cout), _ptr(raw), cap)
        return raw[: min(n, cap) * 32], cout, n

    def decode_indexed(self, buf: np.ndarray, starts):
        st = np.ascontiguousarray(np.asarray(starts, dtype=np.uint64))
        frames = (Frame * max(1, st.size))()
        self.L.oracle_decode_indexed(_ptr(buf), buf.size, _ptr(st), st.size, frames)
        return [frames[i] for i in range(st.size)]

    def digest(self, buf: np.ndarray) -> int:
        return self.L.oracle_digest(_ptr(buf), buf.size)

    def decode_batch_mt(self, buf: np.ndarray, threads: int) -> int:
        """The CPU baseline: serial header walk, threaded unmask (whole frames)."""
        return self.L.oracle_decode_batch_mt(_ptr(buf), buf.size, threads)

    def frames_digest(self, raw: np.ndarray) -> int:
        """Digest of a descriptor table (xyws_frame records as raw bytes): the
        fields the reference defines (offsets, length, key, flags, header
        length) and the PAYLOAD_INCOMPLETE status bit; the informational RFC
        status bits (which the reference does not compute) and the reserved
        byte are masked out."""
        a = np.ascontiguousarray(raw, dtype=np.uint8).reshape(-1, 32).copy()
        a[:, 30] &= 1
        a[:, 31] = 0
        return self.digest(a.reshape(-1))

    # --- callers either side of the path (xyws_frames.hip semantics) ---
    @staticmethod
    def _frames(frames):
        arr = (Frame * max(1, len(frames)))()
        for i, f in enumerate(frames):
            arr[i] = f
        return arr

    def encode_frames(self, src: np.ndarray, frames, flags, enc_opts=0, keys=None, verdicts=None,
                      action_mask=0, out_cap=None):
        """echo_once replies for a frame list: (reply bytes, offsets)."""
        fr = self._frames(frames)
        n = len(frames)
        kb = None if keys is None else np.ascontiguousarray(np.frombuffer(bytes(keys), np.uint8))
        vd = None
        if verdicts is not None:
            vd = (Verdict * max(1, n))()
            for i, v in enumerate(verdicts):
                vd[i] = v
        total = self.L.oracle_encode_frames(_ptr(src), src.size, fr, n, flags, enc_opts, _ptr(kb), vd,
                                            action_mask, None, 0, None)
        cap = total if out_cap is None else out_cap
        out = np.zeros(max(cap, 1), np.uint8)
        offs = np.zeros(n + 1, np.uint64)
        self.L.oracle_encode_frames(_ptr(src), src.size, fr, n, flags, enc_opts, _ptr(kb), vd, action_mask,
                                    _ptr(out), cap, _ptr(offs))
        return out[:min(cap, total)].tobytes(), offs, total

    def classify(self, src: np.ndarray, frames, max_payload, policy):
        n = len(frames)
        fr = self._frames(frames)
        out = (Verdict * max(1, n))()
        first = C.c_uint64()
        self.L.oracle_classify(_ptr(src), src.size, fr, n, max_payload, policy, out, C.byref(first))
        return [out[i] for i in range(n)], first.value

    def utf8_valid(self, data: bytes, complete=True):
        b = np.frombuffer(bytes(data), np.uint8).copy() if data else np.zeros(1, np.uint8)
        return bool(self.L.oracle_utf8_valid(_ptr(b), len(data), 1 if complete else 0))

    def reassemble(self, src: np.ndarray, frames, opts, out_cap=None):
        """(gathered bytes, message list)."""
        n = len(frames)
        fr = self._frames(frames)
        cap_m = max(1, n)
        msgs = (Message * cap_m)()
        total = sum(f.payload_len for f in frames)
        cap = total if out_cap is None else out_cap
        out = np.zeros(max(cap, 1), np.uint8)
        nm = self.L.oracle_reassemble(_ptr(src), src.size, fr, n, opts, _ptr(out), cap, msgs, cap_m)
        return out, [msgs[i] for i in range(nm)]

    def fill_uniform(self, nframes, plen, b0, seed) -> np.ndarray:
        H = 2 + (0 if plen < 126 else (2 if plen <= 0xFFFF else 8)) + 4
        buf = np.empty(nframes * (H + plen), np.uint8)
        self.L.oracle_fill_uniform(_ptr(buf), nframes, plen, b0, seed)
        return buf

    def mixed_table(self, seed, target):
        tot = C.c_uint64()
        n = self.L.oracle_mixed_table(seed, target, None, 0, C.byref(tot))
        tab = (SynthFrame * n)()
        self.L.oracle_mixed_table(seed, target, tab, n, C.byref(tot))
        return tab, n, tot.value

    def fill_mixed(self, tab, n, total, seed) -> np.ndarray:
        buf = np.empty(total, np.uint8)
        self.L.oracle_fill_mixed(_ptr(buf), tab, n, seed)
        return buf


def ref_lib_path(opt="O2"):
    name = "libxynet_ref.so" if opt == "O2" else "libxynet_ref_O0.so"
    return os.path.join(HERE, "_ref", name)


class Reference:
    """The reference's own parser/mask (oracle/_ref), when it was built."""

    def __init__(self, opt="O2"):
        path = ref_lib_path(opt)
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.L = C.CDLL(path)
        u64, u32, u8, vp = C.c_uint64, C.c_uint32, C.c_uint8, C.c_void_p
        L.ref_parser_new.restype = vp
        L.ref_parser_free.argtypes = [vp]
        L.ref_parser_reset.argtypes = [vp]
        L.ref_parser_parse.restype = u64
        L.ref_parser_parse.argtypes = [vp, vp, u64]
        L.ref_parser_result.argtypes = [vp, C.POINTER(u8), C.POINTER(u32), C.POINTER(u64), vp]
        L.ref_mask.restype = u64
        L.ref_mask.argtypes = [vp, u64, u32, u64]
        L.ref_header_build.restype = u64
        L.ref_header_build.argtypes = [vp, u8, vp, u64]
        L.ref_header_ctor.restype = u64
        L.ref_header_ctor.argtypes = [vp, u8, u64]
        L.ref_header_ctor_masked.restype = u64
        L.ref_header_ctor_masked.argtypes = [vp, u8, u32, u64]
        L.ref_calc_frame_header_size.restype = u64
        L.ref_calc_frame_header_size.argtypes = [u8, u64]
        L.ref_decode_stream.restype = u64
        L.ref_decode_stream.argtypes = [vp, u64, vp, vp, vp, u64]
        L.ref_decode_batch_mt.restype = u64
        L.ref_decode_batch_mt.argtypes = [vp, u64, C.c_int]

    class Parser:
        def __init__(self, L):
            self.L = L
            self.h = L.ref_parser_new()

        def __del__(self):
            try:
                self.L.ref_parser_free(self.h)
            except Exception:
                pass

        def parse(self, data: bytes):
            b = C.create_string_buffer(bytes(data), max(len(data), 1))
            return self.L.ref_parser_parse(self.h, b, len(data))

        def reset(self):
            self.L.ref_parser_reset(self.h)

        def result(self):
            f, m, l = C.c_uint8(), C.c_uint32(), C.c_uint64()
            mb = (C.c_uint8 * 4)()
            self.L.ref_parser_result(self.h, C.byref(f), C.byref(m), C.byref(l), mb)
            return f.value, m.value, l.value

    def parser(self):
        return Reference.Parser(self.L)

    def mask(self, arr, key_u32, phase):
        return self.L.ref_mask(_ptr(arr), arr.size, key_u32, phase)

    def header_build(self, flags, mask, length):
        out = np.zeros(16, np.uint8)
        mk = None if mask is None else np.frombuffer(bytes(mask), np.uint8).copy()
        n = self.L.ref_header_build(_ptr(out), flags, _ptr(mk), length)
        return out[:n].tobytes()

    def header_ctor(self, flags, length, mask_u32=None):
        out = np.zeros(16, np.uint8)
        if mask_u32 is None:
            n = self.L.ref_header_ctor(_ptr(out), flags, length)
        else:
            n = self.L.ref_header_ctor_masked(_ptr(out), flags, mask_u32, length)
        return out[:n].tobytes()

    def calc_frame_header_size(self, flags, length):
        return self.L.ref_calc_frame_header_size(flags, length)

    def decode_stream(self, buf, carry_in=None, cap=None):
        n_est = cap if cap is not None else max(16, buf.size // 2 + 2)
        frames = (Frame * n_est)()
        cout = Carry()
        n = self.L.ref_decode_stream(_ptr(buf), buf.size,
                                     C.byref(carry_in) if carry_in is not None else None,
                                     C.byref(cout), frames, n_est)
        return [frames[i] for i in range(min(n, n_est))], cout, n

    def decode_stream_raw(self, buf, cap):
        """decode_stream with the descriptors as one uint8 array (cap * 32 B)."""
        raw = np.zeros(max(cap, 1) * 32, np.uint8)
        cout = Carry()
        n = self.L.ref_decode_stream(_ptr(buf), buf.size, None, C.byref(cout), _ptr(raw), cap)
        return raw[: min(n, cap) * 32], cout, n

    def decode_batch_mt(self, buf, threads):
        return self.L.ref_decode_batch_mt(_ptr(buf), buf.size, threads)
