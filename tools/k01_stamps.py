"""Phase clocks of the class emission launch (diagnostic build lib/libbic_stamps.so, make stamps; the
XSTAMP slots of bic_fused.hip): one C3 encode_gray (the bench's default call, twice), then per wave of
k_emit_k01 its entry / k = 0 rows done / exit (persistent waves) or entry / kmix rows done / exit (rest
role), and per kmix row its entry, loads done and stored times, on the shared 100 MHz clock."""
import json
import os
import sys
import ctypes as C

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BIC_LIB_PATH"] = os.environ.get("STAMPS_LIB") or os.path.join(ROOT, "binary-image-compression_amd", "lib", "libbic_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(0x5EED0000)
rows = cols = 16384
gray = t.randint(0, 256, (rows, cols), dtype=t.uint8, device=ctx.dev, generator=g)
lib = pybic.load()
lib.bic_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
n = 1 << 22
d = lambda a: np.percentile(a, [0, 10, 50, 90, 100]).round(2).tolist() if len(a) else []  # noqa: E731
for rep in range(2):
    buf0 = np.zeros(n, np.uint64)
    assert lib.bic_debug_stamps(buf0.ctypes.data, n) == 0
    ctx.encode_gray(gray, store_planes=False)
    ctx.sync()
    buf = np.zeros(n, np.uint64)
    assert lib.bic_debug_stamps(buf.ctypes.data, n) == 0
    W = buf[((1 << 19) + 8192) * 4:((1 << 19) + 8192 + 8192) * 4].reshape(-1, 4).astype(np.int64)
    W0 = buf0[((1 << 19) + 8192) * 4:((1 << 19) + 8192 + 8192) * 4].reshape(-1, 4).astype(np.int64)
    live = (W[:, 0] > 0) & (W[:, 0] != W0[:, 0])
    t0 = W[live, 0].min()
    K = buf[(1 << 18) * 4:((1 << 18) + rows * 8) * 4].reshape(-1, 4).astype(np.int64)
    K0 = buf0[(1 << 18) * 4:((1 << 18) + rows * 8) * 4].reshape(-1, 4).astype(np.int64)
    km = (K[:, 0] > 0) & (K[:, 0] != K0[:, 0])
    Kk = K[km]
    rg = int(os.environ.get("RG", "1024"))  # rest-role waves (the first rg of the launch's waves)
    idx = np.nonzero(live)[0]
    rest = idx[idx < rg]
    pers = idx[idx >= rg]
    out = dict(rep=rep, waves=int(live.sum()),
               persistent_k0_done_us=d((W[pers, 1] - t0) / 100), persistent_exit_us=d((W[pers, 3] - t0) / 100),
               rest_kmix_done_us=d((W[rest, 1] - t0) / 100), rest_exit_us=d((W[rest, 3] - t0) / 100),
               kmix_rows=int(km.sum()), kmix_start_us=d((Kk[:, 0] - t0) / 100),
               kmix_load_us=d((Kk[:, 1] - Kk[:, 0]) / 100), kmix_code_us=d((Kk[:, 2] - Kk[:, 1]) / 100))
    print(json.dumps(out), flush=True)
    # where the spread comes from: per XCD (block % 8), per wave of the workgroup, per CU slot (block // 8 % ...)
    if rep == 1:
        blk = (idx - 0) // 4
        pw = idx[idx >= rg]
        b = pw // 4
        k0d = (W[pw, 1] - t0) / 100
        ex = (W[pw, 3] - t0) / 100
        st = (W[pw, 0] - t0) / 100
        by = lambda key, v: {int(k): round(float(np.median(v[key == k])), 1) for k in np.unique(key)}  # noqa: E731
        print(json.dumps(dict(start_us=d(st), k0_done_by_xcd=by(b % 8, k0d), exit_by_xcd=by(b % 8, ex),
                              k0_done_by_wave=by(pw % 4, k0d), exit_by_wave=by(pw % 4, ex),
                              k0_done_by_block_third=by(np.minimum(b // (len(b) // 12 + 1), 11), k0d),
                              k1_phase_us=d(ex - k0d), k0_phase_us=d(k0d - st))), flush=True)
    # the k = 1 rows' phases (YSTAMP, issue times): entry -> row assembled (its loads waited for) ->
    # codewords placed in the LDS image -> output stores issued
    if rep == 1:
        K1 = K[(K[:, 0] > 0) & (K[:, 3] > 0) & (K[:, 0] != K0[:, 0])]
        if len(K1):
            print(json.dumps(dict(k1_rows=int(len(K1)), assemble_us=d((K1[:, 1] - K1[:, 0]) / 100),
                                  encode_us=d((K1[:, 2] - K1[:, 1]) / 100), write_us=d((K1[:, 3] - K1[:, 2]) / 100),
                                  total_us=d((K1[:, 3] - K1[:, 0]) / 100))), flush=True)
