"""Decode of the bench's B = 50 latents (256^2): chunking and concurrency variants, GPU time by HIP events (dev tool).
  seq32:  chunks 32 + 18 on one stream (FrozenAutoencoderKL's default)
  seq25:  chunks 25 + 25 on one stream
  lanes2: chunks 25 + 25 on two streams at once (private workspaces)
Usage: python3 tools/decode_lanes.py [B [latent]]"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402
from panopticdiffusionmodels_amd.libs.autoencoder import get_model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 50
S = int(sys.argv[2]) if len(sys.argv) > 2 else 32   # latent size (64: 512^2)
dev = torch.device("cuda")
ae = get_model(None, seed=1, latent_size=S).to(dev)
z = torch.randn(B, 4, S, S, device=dev)
ref = ae.decode(z)
nat = ae.native(dev)
h2 = (B + 1) // 2
wsa, wsb = nat.workspace(max(32, h2)), None
wsb = torch.empty_like(wsa)
img = torch.empty_like(ref)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def dec(lo, hi, ws, stream):
    _lib.check(nat.lib.pdm_decoder_decode(nat.h, _lib.ptr(z[lo:hi]), _lib.ptr(img[lo:hi]), hi - lo, _lib.ptr(ws),
                                          ws.numel(), _lib.ctypes.c_void_p(stream.cuda_stream)), "decode")


def seq(chunk):
    st = torch.cuda.current_stream()
    for s in range(0, B, chunk):
        dec(s, min(B, s + chunk), wsa, st)


def lanes2():
    main = torch.cuda.current_stream()
    s1.wait_stream(main)
    s2.wait_stream(main)
    dec(0, h2, wsa, s1)
    dec(h2, B, wsb, s2)
    main.wait_stream(s1)
    main.wait_stream(s2)


variants = {"seq32": lambda: seq(32), "seq25": lambda: seq(h2), "lanes2": lanes2}
for nm, fn in variants.items():
    fn()
    torch.cuda.synchronize()
    err = float((img - ref).abs().max())
    assert err == 0.0, (nm, err)
t = {k: [] for k in variants}
for _ in range(5):
    for nm, fn in variants.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        t[nm].append(e0.elapsed_time(e1))
print(f"decode B={B} {8 * S}^2: " + "  ".join(f"{k} {sorted(v)[2]:6.2f} ms" for k, v in t.items()) + "  (bit-identical)")
