"""diagnostic: the first encode of a process over poisoned device memory (argv: rows cols mode poison)
-- poison 0: none; 1: 2 GiB of 0xff bytes freed back to the driver before the context's buffers are
made; 2: the same with random bytes; 3: 0xff left in torch's cache (the output tensors)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pybic  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

rows, cols, mode, poison = (int(x) for x in sys.argv[1:5])
o = Oracle()
img = o.gen_bytes(rows * 13 + cols, rows * cols).reshape(rows, cols)
P = o.bitplanes(img, 8)
exp = [o.encode_plane(P[k], cols, 1, 0) for k in range(8)]
import torch  # noqa: E402
dev = torch.device("cuda", 0)
if poison:
    n = 1 << 28
    if poison == 2:
        x = torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=dev)
    else:
        x = torch.full((n,), -1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    if poison == 3:
        xs = [torch.full((1 << 20,), -1, dtype=torch.int64, device=dev) for _ in range(64)]
        del xs
    del x
    if poison != 3:
        torch.cuda.empty_cache()
ctx = pybic.Context(0)
ctx.set_encoder("staged")
ctx.set_eg_source(mode)
g = ctx.torch.from_numpy(img).to(ctx.dev)
_, (og, bg), _ = ctx.encode_gray(g, store_planes=False)
ctx.sync()
bad = [k for k in range(8) if pybic.stream_bytes(og[k], exp[k][0]) != exp[k][1].tobytes()]
print(f"{rows}x{cols} mode {mode} poison {poison}: bad planes {bad}", flush=True)
