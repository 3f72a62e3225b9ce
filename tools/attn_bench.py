"""A/B timing of the attention structures on one U-ViT shape (dev tool, one process, interleaved rounds).
python tools/attn_bench.py [rows L H Dh [algos [q_log2 0|1]]]  (q_log2 1, the default: q pre-scaled as the
U-ViT forward's qkv GEMM writes it, pdm_attention_log2)"""
import sys

import torch

sys.path.insert(0, ".")
from panopticdiffusionmodels_amd import _lib  # noqa: E402

rows, L, H, Dh = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (190, 258, 16, 64)))
lib = _lib.load()
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(rows * L, 3 * H * Dh, device="cuda", generator=g).bfloat16()
flops = 4.0 * rows * H * L * L * Dh
algos = [int(a) for a in sys.argv[5].split(',')] if len(sys.argv) > 5 else [1, 2, 3, 4, 5, 6]
algos = [a for a in algos if lib.pdm_set_attention_algo(a) == 0]   # an A/B build may not know every algo
TIMING_ONLY = (5, 6, 8, 9, 12, 13, 15, 16)   # load-only / math-only variants: wrong results by design
LOG2 = bool(int(sys.argv[6])) if len(sys.argv) > 6 else True
outs = {}
for a in algos:
    assert lib.pdm_set_attention_algo(a) == 0, lib.pdm_last_error()
    outs[a] = _lib.attention(qkv, rows, L, H, Dh, q_log2=LOG2).float()
err = max([float((outs[algos[0]] - outs[a]).norm() / outs[algos[0]].norm()) for a in algos if a not in TIMING_ONLY] + [0.0])
times = {a: [] for a in algos}
for rnd in range(7):
    for a in algos:
        assert lib.pdm_set_attention_algo(a) == 0, lib.pdm_last_error()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            _lib.attention(qkv, rows, L, H, Dh, q_log2=LOG2)
        e1.record()
        torch.cuda.synchronize()
        times[a].append(e0.elapsed_time(e1) / 10)
lib.pdm_set_attention_algo(0)
# vendor reference point: torch SDPA (flash / CK backend) on [rows, H, L, Dh] bf16 views of the same qkv
q, k, v = qkv.view(rows, L, 3, H, Dh).permute(2, 0, 3, 1, 4).contiguous().unbind(0)
ts = []
for rnd in range(7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.nn.functional.scaled_dot_product_attention(q, k, v)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 10)
t_sdpa = sorted(ts)[3]
line = f"attention rows={rows} L={L} H={H} Dh={Dh} maxrelerr={err:.1e} | sdpa {t_sdpa*1e3:8.1f} us {flops/t_sdpa/1e9:7.1f} TF/s"
for a in algos:
    t = sorted(times[a])[3]
    line += f" | algo{a} {t*1e3:8.1f} us {flops/t/1e9:7.1f} TF/s"
print(line)
