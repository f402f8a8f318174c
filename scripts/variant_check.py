"""Debug aid: one config batch decoded ONCE per variant, each on a freshly
generated batch, by the run decoder with the given xopts: frame count and
output digest against the reference's (tests/golden/configs.json).
  usage: variant_check.py NAME XOPTS..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import torch
    from test_gpu_parity import tools_batch, dev_digest
    from xynet_amd import _lib, websocket as ws
    name = sys.argv[1]
    for xs in sys.argv[2:]:
        x = int(xs, 0)
        buf, c = tools_batch(name)
        dec = ws.frame_decoder(opts=_lib.OPT_RUNS | x)
        r = dec.decode(buf, cap=0, count=True, carry=False)
        n = r.nframes
        ok = dev_digest(buf) == c["out_digest"]
        print(name, xs, "frames", n, "expected", c["decoded_frames"], "digest_ok", ok, "err",
              dec.ctx.last_device_error(), flush=True)
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
