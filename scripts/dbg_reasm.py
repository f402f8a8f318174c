"""Debug aid (round 6): xyws_reassemble's records against the oracle's on one
message stream, every differing message printed with the frames around it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import msg_streams
    from oracle.oracle import Oracle
    from test_frames import _decode, _messages
    from xynet_amd import _lib
    from xynet_amd import websocket as ws
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    oracle = Oracle()
    wire, _ = msg_streams.message_stream(seed, nmsg=80)
    t, frames_t, n, host, ofr = _decode(ws, oracle, wire)
    oout, orecs = oracle.reassemble(host, ofr, _lib.REASM_UTF8)
    out, mt, cnt = ws.reassemble(t, frames_t, n, _lib.REASM_UTF8)
    nm = int(cnt.item())
    got = _messages(mt, nm)
    want = [r.as_tuple() for r in orecs]
    print("frames", n, "messages", nm, len(want))
    ops = [(i, f.flags & 0xF, (f.flags >> 4) & 1) for i, f in enumerate(ofr)]
    for m, (g, w) in enumerate(zip(got, want)):
        if g != w:
            s = w[0]
            print("msg", m, "got", g, "want", w)
            print("   frames", ops[max(0, s - 6):s + 2])


if __name__ == "__main__":
    main()
