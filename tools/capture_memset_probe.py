"""Diagnostic: is a hipMemsetAsync enqueued under stream capture (bic_memset inside torch.cuda.graph)
replayed as a memset of the same bytes? Fills a buffer with 0x55, replays, reports the zeroed range."""
import ctypes as C
import sys

sys.path.insert(0, "binary-image-compression_amd")
import torch  # noqa: E402
import pybic  # noqa: E402

ctx = pybic.Context(0)
lib = pybic.load()
buf = torch.empty(1 << 16, dtype=torch.uint8, device=ctx.dev)
for off, n in ((0, 1280), (256, 1024), (0, 8), (4, 4), (0, 4096 + 256), (8, 40000)):
    side = torch.cuda.Stream(ctx.dev)
    side.wait_stream(torch.cuda.current_stream(ctx.dev))
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(gr, stream=side):
            ctx._bind_stream()
            assert lib.bic_memset(ctx.h, C.c_void_p(buf.data_ptr() + off), 0, n) == 0
    torch.cuda.current_stream(ctx.dev).wait_stream(side)
    torch.cuda.synchronize()
    buf.fill_(0x55)
    torch.cuda.synchronize()
    ctx._bind_stream()
    gr.replay()
    torch.cuda.synchronize()
    z = (buf == 0).nonzero().flatten()
    print({"off": off, "n": n, "zeroed": int(z.numel()), "first": int(z[0]) if z.numel() else None,
           "last": int(z[-1]) if z.numel() else None}, flush=True)
