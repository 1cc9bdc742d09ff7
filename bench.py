"""bench.py -- encode throughput of the MI355X hot path (BASELINE.json metric:
"encode MPixels/s (and MB/s out) at 1/2/4/8 GPUs; bit-exact vs CPU").

Default workload (c3, BASELINE.json configs[2], the north star's roofline config): per GPU one
16384x16384 8-bit gray image (synthetic, device-resident) -> 8 bitplanes -> med residual ->
per-row runs -> Golomb stream AND EG stream for every plane. MPix = binary pixels =
rows*cols*planes. N GPUs = N independent images (weak scaling, no data-path collective).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]

Multi-GPU: one rank per GPU (RCCL = backend "nccl"). Under torch.distributed.run (WORLD_SIZE set) this
process is one rank; `bench.py --gpus N` without a launcher starts the N ranks itself, as a child
torch.distributed.run of the same command, and exits with its code. Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "encode MPixels/s (and MB/s out) at 1/2/4/8 GPUs; bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=["c1", "c1m", "c2", "c3", "c3f", "c4", "c5"])
    ap.add_argument("--rows", type=int, default=0, help="override image rows (c3/c2/c5)")
    ap.add_argument("--cols", type=int, default=0, help="override image cols")
    ap.add_argument("--cpu-rows", type=int, default=16384, help="rows per plane in the CPU baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="repeat the CPU baseline sample until this much CPU time has been measured")
    ap.add_argument("--encoder", default="auto", choices=["auto", "staged", "single-kernel", "two-pass", "multipass"],
                    help="row encoder for rows <= 16384 columns (bic_ctx_set_option)")
    ap.add_argument("--one-stream", action="store_true",
                    help="diagnostic: the staged encoder's two emission launches one after the other on one stream")
    ap.add_argument("--shard", default="images", choices=["images", "planes"],
                    help="c3 at N GPUs: one image per GPU (weak scaling, no exchange) or the 8 planes of ONE "
                         "image split over the GPUs, every rank's packed streams gathered to rank 0 over RCCL "
                         "(strong scaling; the gather is in the timed step)")
    ap.add_argument("--separate", action="store_true",
                    help="c3: bic_bitplanes_u8 then bic_encode_planes2 instead of the one-call bic_encode_gray")
    ap.add_argument("--store-planes", action="store_true",
                    help="c3: bic_encode_gray also returns the 8 bitplanes (planes != NULL; +256 MiB written per "
                         "image); default: planes NULL, the count pass keeps the residual planes for the encoder")
    ap.add_argument("--eg-source-mode", type=int, default=1,
                    help="BIC_OPT_EG_SOURCE value when the EG source is on (1: row-class kernels, 2: one kernel)")
    ap.add_argument("--no-eg-source", action="store_true",
                    help="c3 (planes NULL): the round-3 path -- the count pass stores the med residual planes for "
                         "the encoder -- instead of writing the EG stream and reading the residual rows back from it")
    ap.add_argument("--plane-count", type=int, default=8,
                    help="c3 --shard planes: encode planes 0..P-1 of the image (split over the ranks); P = 1 or 2 at "
                         "N = 1 measures the per-rank step of a plane-sharded 8- or 4-GPU run")
    ap.add_argument("--chunks", type=int, default=0,
                    help="c4 / c3 --shard planes at N > 1: encode a rank's units in this many chunks, each chunk's "
                         "streams sent to rank 0 while the next encodes (pybic.parallel.ChunkedGather); 0 = auto "
                         "(2 for c4, 1 per plane for --shard planes), 1 = one gather after the encode")
    ap.add_argument("--inflight", type=int, default=1,
                    help="c3 (one-call, planes NULL): images in flight -- this many contexts, each on its own HIP "
                         "stream, take successive images, so one image's emission overlaps the next one's count "
                         "pass (serving throughput; the roofline kernel is timed on the first context's launches)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    return ap.parse_args()


def spawn_ranks(args):
    """`bench.py --gpus N` (N > 1) started without a launcher: run N ranks of this same command
    under torch.distributed.run as a CHILD process (never exec) before anything here touches the
    GPU, and return its exit code. Under a launcher (WORLD_SIZE set) this returns None and the
    process is one rank."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8")))


def dist_setup(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BIC_BENCH_BACKEND=gloo rehearses the N-rank path with several ranks on one GPU (functional
    # check only); the real run is one rank per GPU over RCCL (backend "nccl")
    backend = os.environ.get("BIC_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def barrier(world):
    import torch
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        torch.cuda.synchronize()


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_i64(vals, world, dev):
    """every rank's list of ints (same length on every rank), in rank order"""
    if world == 1:
        return [list(vals)]
    import torch
    import torch.distributed as dist
    host = dist.get_backend() == "gloo"
    t = torch.tensor(list(vals), dtype=torch.int64, device="cpu" if host else dev)
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return [o.cpu().tolist() for o in outs]


def checksum(t):
    """order-independent 64-bit fingerprint of a device tensor's words (wrapping sum and xor)"""
    import torch
    w = t.reshape(-1).view(torch.int64)
    x = w.clone()
    n = x.numel()
    while n > 1:  # xor-reduce by halves (torch has no xor reduction)
        h = n // 2
        x[:h] ^= x[n - h:n]
        n -= h
    return [int(w.sum().item()), int(x[0].item()) if x.numel() else 0]


def sum_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def load_pmc(workload, kernel):
    """(HBM bytes per launch, note) from the newest round's committed rocprofv3 PMC summary
    (profiles/rNN/pmc_<workload>.json). The summary carries the hash of the kernel sources it
    profiled (pybic.sources_hash): a summary of other sources than the ones built here does not
    describe this run's kernels, so it gives no traffic (None) and a note saying so."""
    import pybic
    got = _load_pmc(workload, kernel)
    if got is None:
        return None, "no PMC summary for this workload"
    v, path, src = got
    if src != pybic.sources_hash():
        print(f"bench.py: {path} profiled other kernel sources ({src}); roofline.traffic left null",
              file=sys.stderr)
        return None, f"{os.path.relpath(path, ROOT)} profiled other kernel sources: traffic not reported"
    return v, f"{os.path.relpath(path, ROOT)} (PMC FETCH_SIZE/WRITE_SIZE passes of these kernel sources)"


def _load_pmc(workload, kernel):
    pdir = os.path.join(ROOT, "profiles")
    try:
        rounds = sorted((d for d in os.listdir(pdir) if d.startswith("r") and d[1:].isdigit()), reverse=True)
    except OSError:
        return None
    for r in rounds:
        path = os.path.join(pdir, r, f"pmc_{workload}.json")
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        for sec in ("timers", "kernels"):
            v = d.get(sec, {}).get(kernel, {}).get("hbm_bytes_per_launch")
            if v is not None:
                return v, path, d.get("sources_sha256")
        return None
    return None


def rand_words(t, shape, dev, g):
    """uniform 64-bit words (Bernoulli(0.5) pixels) as int64, generated on the device."""
    n = int(np.prod(shape))
    return t.randint(0, 256, (n * 8,), dtype=t.uint8, device=dev, generator=g).view(t.int64).view(*shape)


# ------------------------------------------------------------------------------------------
class C3:
    """gray image -> 8 bitplanes -> med -> Golomb + EG (per GPU)."""

    def __init__(self, ctx, args, rank):
        import pybic
        t = ctx.torch
        self.ctx, self.pybic = ctx, pybic
        self.rows = args.rows or 16384
        self.cols = args.cols or 16384
        self.nplanes = 8
        g = t.Generator(device=ctx.dev)
        g.manual_seed(0x5EED0000 + rank)
        # two gray buffers, alternated per step, so the Infinity Cache cannot serve re-runs
        self.inflight = max(1, args.inflight)
        self.gray = [t.randint(0, 256, (self.rows, self.cols), dtype=t.uint8, device=ctx.dev, generator=g)
                     for _ in range(max(2, self.inflight))]
        self.wpr = (self.cols + 63) // 64
        self.separate = args.separate
        self.store_planes = args.store_planes or args.separate
        # planes NULL: the count pass writes the EG stream and the Golomb emission reads the residual rows
        # from it (BIC_OPT_EG_SOURCE; off: the residual planes stored in a context buffer)
        self.eg_src = not self.store_planes and not args.no_eg_source
        ctx.set_eg_source(args.eg_source_mode if self.eg_src else 0)
        self.planes = ctx.empty_i64(self.nplanes, self.rows, self.wpr) if self.store_planes else None
        self.slot_g = ctx.slot_words(self.rows, self.cols, pybic.CODER_GOLOMB)
        self.slot_e = ctx.slot_words(self.rows, self.cols, pybic.CODER_EG)
        self.out_g = ctx.empty_i64(self.nplanes, self.slot_g)
        self.out_e = ctx.empty_i64(self.nplanes, self.slot_e)
        self.bits_g = ctx.empty_i64(self.nplanes)
        self.bits_e = ctx.empty_i64(self.nplanes)
        ctx.reserve(self.nplanes, self.rows, self.cols)
        self.lanes = None
        if self.inflight > 1:
            # images in flight: context i (its own stream, aux stream and scratch) encodes images k = i mod n;
            # one context per stream (include/bic.h), outputs per context
            if self.separate or self.store_planes:
                raise SystemExit("--inflight needs the one-call encode with planes NULL")
            self.lanes = [(ctx, t.cuda.Stream(ctx.dev), self.out_g, self.out_e, self.bits_g, self.bits_e)]
            for _ in range(self.inflight - 1):
                c = pybic.Context(ctx.dev.index)
                c.set_encoder(args.encoder)
                c.set_eg_source(args.eg_source_mode if self.eg_src else 0)
                c.reserve(self.nplanes, self.rows, self.cols)
                self.lanes.append((c, t.cuda.Stream(ctx.dev), c.empty_i64(self.nplanes, self.slot_g),
                                   c.empty_i64(self.nplanes, self.slot_e), c.empty_i64(self.nplanes),
                                   c.empty_i64(self.nplanes)))
        self.k = 0
        self.pixels = self.rows * self.cols * self.nplanes
        self.workload = (f"c3: {self.rows}x{self.cols} 8-bit gray -> 8 bitplanes -> med -> per-row runs "
                         f"-> Golomb + EG streams per plane" +
                         ("" if self.store_planes else " (bitplanes formed in registers, not returned: planes NULL)") +
                         (" -- the count pass writes the EG stream, the Golomb emission reads the residual rows "
                          "from it" if self.eg_src else "") +
                         (f" -- {self.inflight} images in flight (one context and HIP stream each)"
                          if self.inflight > 1 else ""))

    def step(self):
        c = self.ctx
        if self.lanes:
            i = self.k % self.inflight
            c, s, self.out_g, self.out_e, self.bits_g, self.bits_e = self.lanes[i]  # the last step's outputs
            with self.ctx.torch.cuda.stream(s):
                c.encode_gray(self.gray[i], nplanes=8, planes=None, slots=(self.slot_g, self.slot_e),
                              outs=(self.out_g, self.out_e), bits=(self.bits_g, self.bits_e), store_planes=False)
        elif self.separate:
            c.bitplanes_u8(self.gray[self.k % len(self.gray)], nplanes=8, out=self.planes)
            c.encode_planes2(self.planes, self.cols, True, slots=(self.slot_g, self.slot_e),
                             outs=(self.out_g, self.out_e), bits=(self.bits_g, self.bits_e))
        else:  # one call: bitplanes + both streams (bic_encode_gray)
            c.encode_gray(self.gray[self.k % len(self.gray)], nplanes=8, planes=self.planes, slots=(self.slot_g, self.slot_e),
                          outs=(self.out_g, self.out_e), bits=(self.bits_g, self.bits_e),
                          store_planes=self.store_planes)
        self.k += 1

    def out_bytes(self):
        b = self.pybic.as_u64(self.bits_g).astype(np.int64).sum() + self.pybic.as_u64(self.bits_e).astype(np.int64).sum()
        return int(b) / 8.0

    def kernel_bytes(self):
        """algorithmic bytes per launch."""
        plane_b = self.nplanes * self.rows * self.wpr * 8
        g = int(self.pybic.as_u64(self.bits_g).astype(np.int64).sum()) // 8
        e = int(self.pybic.as_u64(self.bits_e).astype(np.int64).sum()) // 8
        # EG source: the count pass writes the EG stream (not R) and the emission reads it and writes Golomb
        return {"bitplanes_u8": self.rows * self.cols + plane_b,
                "bitplanes_count": self.rows * self.cols + (e if self.eg_src else plane_b),
                "med_count": plane_b, "golomb_bits": plane_b,
                "golomb_emit": plane_b + g, "eg_emit": plane_b + e, "encode_rows_golomb_eg": plane_b + g + e,
                "encode_rows_golomb_egsrc": e + g}

    def host_planes(self, rows):
        if self.planes is None:  # the last step's image's planes (device bitplane kernel), for the CPU leg
            return self.pybic.as_u64(self.ctx.bitplanes_u8(self.gray[(self.k - 1) % len(self.gray)][:rows], nplanes=self.nplanes))
        return self.pybic.as_u64(self.planes[:, :rows])

    def predictor_pass(self, reps):
        """The predictor + run-length pass on its own (BASELINE.json north star: >= 50 % of the HBM
        roofline for 16384x16384x8): med residual of every plane, per-row 1-counts (the run
        counts) and plane weights -- bic_med_residual without storing the residual. Reads the
        planes once; not part of `value`. Two plane buffers (the planes of the two gray images)
        alternate, so the 256 MB Infinity Cache cannot hold the input of the next launch
        (SURVEY.md §8 d)."""
        alt = self.ctx.bitplanes_u8(self.gray[self.k % len(self.gray)], nplanes=8)  # the other image's planes
        cur = self.planes if self.planes is not None else self.ctx.bitplanes_u8(self.gray[(self.k - 1) % len(self.gray)], nplanes=8)
        bufs = [cur, alt]
        self.ctx.sync()
        self.ctx.prof_enable(True)
        for i in range(reps):
            self.ctx.med_residual(bufs[i & 1], self.cols, True, want_resid=False)
        self.ctx.sync()
        prof = self.ctx.prof_collect()
        self.ctx.prof_enable(False)
        del alt, cur, bufs
        n, ms = prof["med_count"]
        avg_s = ms / 1e3 / n
        byts = self.nplanes * self.rows * self.wpr * 8
        return {"kernel": "med_count (k_med_rows + k_plane_weight)", "algorithmic_bytes_per_launch": byts,
                "achieved": round(byts / avg_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(byts / avg_s / 1e9 / HBM_PEAK_GBS, 4), "avg_launch_us": round(avg_s * 1e6, 2),
                "input": "two plane buffers (2 x 256 MiB) alternated"}

    def check(self, oracle):
        """every plane of the last step: the planes (when returned) == the oracle's bitplanes of the
        gray image, and each plane's Golomb and EG streams == the oracle's streams of those bitplanes
        (host threads)"""
        gray = self.gray[(self.k - 1) % len(self.gray)].cpu().numpy()
        P = oracle.bitplanes_par(gray, self.nplanes)
        if self.planes is not None and not np.array_equal(self.pybic.as_u64(self.planes), P):
            return False
        exp = oracle.encode_planes_par(P, self.cols, 1)
        ok = True
        for coder, out, bits in ((0, self.out_g, self.bits_g), (1, self.out_e, self.bits_e)):
            B = self.pybic.as_u64(bits)
            for k in range(self.nplanes):
                eb, est = exp[(k, coder)]
                ok &= int(B[k]) == eb and self.pybic.stream_bytes(out[k], eb) == est.tobytes()
        return bool(ok)


class C3Planes(C3):
    """C3 sharded by planes (SURVEY.md §8 e: "8 planes -> 1 per GPU"): every rank holds the same
    gray image and encodes planes [8r/N, 8(r+1)/N) of it (bic_encode_gray_range), packs each
    coder's streams word-aligned (bic_pack_streams) and sends them to rank 0 (gather_streams: one
    all-gather of sizes, point-to-point RCCL transfers over xGMI), which ends the step holding the
    whole image's streams in plane order. Strong scaling: one image per step whatever N."""

    def __init__(self, ctx, args, rank, world):
        import pybic
        t = ctx.torch
        self.ctx, self.pybic, self.rank, self.world = ctx, pybic, rank, world
        self.rows = args.rows or 16384
        self.cols = args.cols or 16384
        self.total_planes = max(1, min(8, args.plane_count))
        P = self.total_planes
        self.lo, self.hi = rank * P // world, (rank + 1) * P // world
        self.nplanes = self.hi - self.lo
        g = t.Generator(device=ctx.dev)
        g.manual_seed(0x5EED0000)  # the same image on every rank
        self.gray = [t.randint(0, 256, (self.rows, self.cols), dtype=t.uint8, device=ctx.dev, generator=g)
                     for _ in range(2)]
        self.wpr = (self.cols + 63) // 64
        self.store_planes = args.store_planes
        self.planes = ctx.empty_i64(max(1, self.nplanes), self.rows, self.wpr) if self.store_planes else None
        self.slot_g = ctx.slot_words(self.rows, self.cols, pybic.CODER_GOLOMB)
        self.slot_e = ctx.slot_words(self.rows, self.cols, pybic.CODER_EG)
        n = max(1, self.nplanes)
        self.out_g, self.out_e = ctx.empty_i64(n * self.slot_g), ctx.empty_i64(n * self.slot_e)  # packed
        self.bits_g, self.bits_e = ctx.empty_i64(n), ctx.empty_i64(n)
        # a rank with no plane (N > P) sends an empty stream: its offsets stay zero
        self.off_g, self.off_e = (ctx.torch.zeros(n + 1, dtype=t.int64, device=ctx.dev) for _ in range(2))
        self.gathered = (None, None)
        # overlapped gather (N > 1): the rank's planes in chunks (default one per plane), each chunk's
        # packed streams sent while the next chunk encodes
        # (the same chunk count on every rank, empty chunks where a rank has fewer planes: one all-gather
        # per chunk -- pybic.parallel.plan_chunks)
        from pybic.parallel import plan_chunks
        self.chunks = plan_chunks(self.nplanes, P, world, args.chunks) if world > 1 else [(0, self.nplanes)]
        self.chunk_off = [[ctx.torch.zeros(b - a + 1, dtype=t.int64, device=ctx.dev) for _ in range(2)]
                          for a, b in self.chunks]
        ctx.reserve(n, self.rows, self.cols)
        self.k = 0
        self.separate = False
        self.pixels = self.rows * self.cols * self.nplanes
        self.workload = (f"c3 sharded by planes: one {self.rows}x{self.cols} 8-bit gray image per step, its {P} "
                         f"plane(s) split over {world} GPU(s) -> med -> Golomb + EG, packed streams gathered to "
                         f"rank 0")

    def step(self):
        from pybic.parallel import ChunkedGather, gather_streams
        c = self.ctx
        if self.world > 1 and len(self.chunks) > 1:
            cgs = (ChunkedGather(c.dev, self.world, self.rank), ChunkedGather(c.dev, self.world, self.rank))
            for (a, b), (fg, fe) in zip(self.chunks, self.chunk_off):
                rg = self.out_g[a * self.slot_g:b * self.slot_g]
                re = self.out_e[a * self.slot_e:b * self.slot_e]
                if b == a:  # an empty chunk (this rank holds fewer planes than the plan's chunk count)
                    cgs[0].add(rg, 0)
                    cgs[1].add(re, 0)
                    continue
                c.encode_gray_packed(self.gray[self.k & 1], nplanes=b - a, plane0=self.lo + a,
                                     planes=None if self.planes is None else self.planes[a:b],
                                     slots=(self.slot_g, self.slot_e), outs=(rg, re),
                                     bits=(self.bits_g[a:b], self.bits_e[a:b]), offs=(fg, fe),
                                     store_planes=self.store_planes)
                cgs[0].add(rg, fg[-1:])
                cgs[1].add(re, fe[-1:])
            self.gathered = (cgs[0].finish(), cgs[1].finish())
            self.k += 1
            return
        if self.nplanes:  # both streams written packed (word-aligned, plane order): the gather sends them as is
            c.encode_gray_packed(self.gray[self.k & 1], nplanes=self.nplanes, plane0=self.lo, planes=self.planes,
                                 slots=(self.slot_g, self.slot_e), outs=(self.out_g, self.out_e),
                                 bits=(self.bits_g, self.bits_e), offs=(self.off_g, self.off_e),
                                 store_planes=self.store_planes)
        got = []
        for packed, off in ((self.out_g, self.off_g), (self.out_e, self.off_e)):
            if self.world > 1:
                got.append(gather_streams(packed, off[-1:], self.world, self.rank))
            else:
                got.append((packed, off))  # (no host sync in the step: the check reads the total)
        self.gathered = tuple(got)
        self.k += 1

    def collect(self):
        """every rank's per-plane bit counts on every rank (collective, after the timed steps)"""
        import torch
        res = []
        for bits in (self.bits_g, self.bits_e):
            t = torch.zeros(8, dtype=torch.int64)
            t[:self.nplanes] = bits[:self.nplanes].cpu()
            if self.world > 1:
                import torch.distributed as dist
                host = dist.get_backend() == "gloo"
                t = t if host else t.to(self.ctx.dev)
                outs = [torch.zeros_like(t) for _ in range(self.world)]
                dist.all_gather(outs, t)
                res.append([o.cpu().numpy().view(np.uint64) for o in outs])
            else:
                res.append([t.numpy().view(np.uint64)])
        self.allbits = res

    def out_bytes(self):
        b = self.pybic.as_u64(self.bits_g[:self.nplanes]).astype(np.int64).sum() + \
            self.pybic.as_u64(self.bits_e[:self.nplanes]).astype(np.int64).sum()
        return int(b) / 8.0

    def host_planes(self, rows):
        if self.planes is None:
            return self.pybic.as_u64(self.ctx.bitplanes_u8(self.gray[(self.k - 1) & 1][:rows], nplanes=self.nplanes,
                                                           plane0=self.lo))
        return self.pybic.as_u64(self.planes[:self.nplanes, :rows])

    def check(self, oracle):
        """rank 0, after collect(): the gathered streams of all 8 planes == the oracle's streams of
        bitplane_tool's planes of the last step's image"""
        gray = self.gray[(self.k - 1) & 1].cpu().numpy()
        P = self.total_planes
        exp_planes = oracle.bitplanes_par(gray, P)
        exp = oracle.encode_planes_par(exp_planes, self.cols, 1)
        ok = True
        for coder in (0, 1):
            words, offs = self.gathered[coder]
            if self.world == 1:
                offs = [0, int(self.pybic.as_u64(offs)[-1])]
            W = self.pybic.as_u64(words)
            for r in range(self.world):
                a, b = r * P // self.world, (r + 1) * P // self.world
                o = offs[r]
                for k in range(a, b):
                    nb = int(self.allbits[coder][r][k - a])
                    nw = (nb + 63) // 64
                    eb, est = exp[(k, coder)]
                    ok &= nb == eb and W[o:o + nw].tobytes() == est.tobytes()
                    o += nw
                ok &= o == offs[r + 1]
        return bool(ok)

    def kernel_bytes(self):
        plane_b = self.nplanes * self.rows * self.wpr * 8
        g = int(self.pybic.as_u64(self.bits_g[:self.nplanes]).astype(np.int64).sum()) // 8
        e = int(self.pybic.as_u64(self.bits_e[:self.nplanes]).astype(np.int64).sum()) // 8
        return {"bitplanes_count": self.rows * self.cols + plane_b, "encode_rows_golomb_eg": plane_b + g + e}


class C3File(C3):
    """C3 from a P5 file's bytes: the whole file -- header + 16384^2 raster -- is
    resident in HBM as read; a step parses the header on the host (bic_pnm_parse_header, from the
    file's first bytes) and encodes the raster where it lies (19 bytes into the file) in one call:
    bic_encode_gray, whose count pass reads misaligned rows through aligned 16-byte chunks (planes
    NULL, as the default C3 step). --separate: bic_pgm_bitplanes then bic_encode_planes2."""

    def __init__(self, ctx, args, rank):
        import pybic
        t = ctx.torch
        self.ctx, self.pybic = ctx, pybic
        self.rows = args.rows or 16384
        self.cols = args.cols or 16384
        self.nplanes = 8
        g = t.Generator(device=ctx.dev)
        g.manual_seed(0x5EED0000 + rank)
        hdr = f"P5\n{self.cols} {self.rows}\n255\n".encode()
        self.head = hdr + b"\0" * 45  # the host's copy of the file's first bytes
        self.files = []
        for _ in range(2):  # two files alternated (the Infinity Cache cannot serve a re-run)
            f = t.empty(len(hdr) + self.rows * self.cols, dtype=t.uint8, device=ctx.dev)
            f[:len(hdr)] = t.tensor(list(hdr), dtype=t.uint8)
            f[len(hdr):] = t.randint(0, 256, (self.rows * self.cols,), dtype=t.uint8, device=ctx.dev, generator=g)
            self.files.append(f)
        self.gray = [f[len(hdr):].view(self.rows, self.cols) for f in self.files]
        self.wpr = (self.cols + 63) // 64
        self.separate = args.separate
        self.store_planes = args.separate or args.store_planes
        self.eg_src = not self.store_planes and not args.no_eg_source
        ctx.set_eg_source(args.eg_source_mode if self.eg_src else 0)
        self.planes = ctx.empty_i64(self.nplanes, self.rows, self.wpr) if self.store_planes else None
        self.slot_g = ctx.slot_words(self.rows, self.cols, pybic.CODER_GOLOMB)
        self.slot_e = ctx.slot_words(self.rows, self.cols, pybic.CODER_EG)
        self.out_g = ctx.empty_i64(self.nplanes, self.slot_g)
        self.out_e = ctx.empty_i64(self.nplanes, self.slot_e)
        self.bits_g = ctx.empty_i64(self.nplanes)
        self.bits_e = ctx.empty_i64(self.nplanes)
        ctx.reserve(self.nplanes, self.rows, self.cols)
        self.k = 0
        self.pixels = self.rows * self.cols * self.nplanes
        self.workload = (f"c3f: a {self.rows}x{self.cols} P5 file's bytes in HBM -> header (host) -> 8 bitplanes "
                         f"from the raster in place (offset {len(hdr)}) -> med -> Golomb + EG streams per plane" +
                         (" (bic_pgm_bitplanes + bic_encode_planes2)" if self.separate else
                          " (one bic_encode_gray call on the misaligned raster)"))

    def step(self):
        c = self.ctx
        h = self.pybic.pnm_header(self.head)
        f = self.files[self.k & 1]
        if self.separate or h.maxval > 255:
            c.pgm_bitplanes(f[h.data_offset:], h.rows, h.cols, h.maxval, self.nplanes, out=self.planes)
            c.encode_planes2(self.planes, self.cols, True, slots=(self.slot_g, self.slot_e),
                             outs=(self.out_g, self.out_e), bits=(self.bits_g, self.bits_e))
        else:  # 8-bit samples: the raster is a gray image with pitch = cols, wherever it starts
            raster = f[h.data_offset:h.data_offset + h.rows * h.cols].view(h.rows, h.cols)
            c.encode_gray(raster, cols=h.cols, nplanes=8, planes=self.planes, slots=(self.slot_g, self.slot_e),
                          outs=(self.out_g, self.out_e), bits=(self.bits_g, self.bits_e),
                          store_planes=self.store_planes)
        self.k += 1

    def kernel_bytes(self):
        kb = super().kernel_bytes()
        kb["pgm_bitplanes"] = kb["bitplanes_u8"]
        return kb


class C2(C3):
    """one 4096x4096 bitplane, Golomb on the raw plane (no predictor)."""

    def __init__(self, ctx, args, rank):
        import pybic
        t = ctx.torch
        self.ctx, self.pybic = ctx, pybic
        self.rows = args.rows or 4096
        self.cols = args.cols or 4096
        self.nplanes = 1
        self.wpr = (self.cols + 63) // 64
        g = t.Generator(device=ctx.dev)
        g.manual_seed(0x5EED0000 + rank)
        self.planes_in = [rand_words(t, (1, self.rows, self.wpr), ctx.dev, g) for _ in range(2)]
        self.planes = self.planes_in[0]
        self.slot_g = ctx.slot_words(self.rows, self.cols, pybic.CODER_GOLOMB)
        self.out_g = ctx.empty_i64(1, self.slot_g)
        self.bits_g = ctx.empty_i64(1)
        self.out_e, self.bits_e = None, ctx.torch.zeros(1, dtype=t.int64, device=ctx.dev)
        ctx.reserve(1, self.rows, self.cols)
        self.k = 0
        self.pixels = self.rows * self.cols
        self.workload = f"c2: one {self.rows}x{self.cols} bitplane, Golomb-only (raw runs, no predictor)"

    def step(self):
        self.planes = self.planes_in[self.k & 1]
        self.ctx.encode_planes(self.planes, self.cols, False, self.pybic.CODER_GOLOMB, self.slot_g, self.out_g,
                               self.bits_g)
        self.k += 1

    def kernel_bytes(self):
        plane_b = self.rows * self.wpr * 8
        g = int(self.pybic.as_u64(self.bits_g)[0]) // 8
        return {"med_count": plane_b, "golomb_bits": plane_b, "golomb_emit": plane_b + g,
                "encode_rows_golomb": plane_b + g}

    def check(self, oracle):
        P = self.pybic.as_u64(self.planes[0])
        eb, est, _ = oracle.encode_plane(P, self.cols, 0, 0)
        nb = int(self.pybic.as_u64(self.bits_g)[0])
        return nb == eb and self.pybic.stream_bytes(self.out_g[0], nb) == est.tobytes()


class C4(C3):
    """64 independent 4096x4096 frames sharded over the ranks (strong scaling), med + Golomb,
    streams packed per rank and gathered to rank 0 over RCCL."""

    TOTAL = 64

    def __init__(self, ctx, args, rank, world):
        import pybic
        t = ctx.torch
        self.ctx, self.pybic, self.rank, self.world = ctx, pybic, rank, world
        self.rows = args.rows or 4096
        self.cols = args.cols or 4096
        self.nplanes = len(self.share(rank))
        self.wpr = (self.cols + 63) // 64
        self.planes = self.frames_of(rank)
        self.slot_g = ctx.slot_words(self.rows, self.cols, pybic.CODER_GOLOMB)
        self.out_g = ctx.empty_i64(max(1, self.nplanes), self.slot_g)
        self.bits_g = ctx.torch.zeros(max(1, self.nplanes), dtype=t.int64, device=ctx.dev)
        self.bits_e = ctx.torch.zeros(1, dtype=t.int64, device=ctx.dev)
        self.packed = ctx.empty_i64(max(1, self.nplanes) * self.slot_g)  # the streams, word-aligned back to back
        self.word_off = ctx.torch.zeros(self.nplanes + 1, dtype=t.int64, device=ctx.dev)
        self.gathered = (None, None)
        # overlapped gather (N > 1): the rank's frames in chunks, each chunk's packed streams in its own
        # region of `packed`, sent while the next chunk encodes
        from pybic.parallel import plan_chunks
        self.chunks = plan_chunks(self.nplanes, self.TOTAL, world, args.chunks or 2) if world > 1 else [(0, self.nplanes)]
        self.chunk_off = [ctx.torch.zeros(b - a + 1, dtype=t.int64, device=ctx.dev) for a, b in self.chunks]
        ctx.reserve(max(1, self.nplanes), self.rows, self.cols)
        self.k = 0
        self.pixels = self.rows * self.cols * self.nplanes
        self.workload = (f"c4: 64 frames {self.rows}x{self.cols} sharded over ranks, med -> Golomb, "
                         f"per-rank packed streams gathered to rank 0 (RCCL)")

    def share(self, r):
        return range(r * self.TOTAL // self.world, (r + 1) * self.TOTAL // self.world)

    def frames_of(self, r):
        """rank r's frames (seeded per rank on the device: rank 0 regenerates any rank's for the check)"""
        t = self.ctx.torch
        g = t.Generator(device=self.ctx.dev)
        g.manual_seed(0x5EED0000 + r)
        return rand_words(t, (max(1, len(self.share(r))), self.rows, self.wpr), self.ctx.dev, g)

    def step(self):
        from pybic.parallel import ChunkedGather, gather_streams
        c = self.ctx
        # packed output: the encoder writes each frame's stream at its packed word offset (no slots, no
        # pack kernel), ready for the gather
        if self.world > 1 and len(self.chunks) > 1:
            cg = ChunkedGather(c.dev, self.world, self.rank)
            for (a, b), off in zip(self.chunks, self.chunk_off):
                if b > a:
                    region = self.packed[a * self.slot_g:b * self.slot_g]
                    c.encode_planes_packed(self.planes[a:b], self.cols, True, golomb=True, eg=False,
                                           slots=(self.slot_g, None), outs=(region, None),
                                           bits=(self.bits_g[a:b], None), offs=(off, None))
                    cg.add(region, off[-1:])
                else:
                    cg.add(self.packed[:0], 0)
            self.gathered = cg.finish()
        else:
            if self.nplanes:
                c.encode_planes_packed(self.planes[:self.nplanes], self.cols, True, golomb=True, eg=False,
                                       slots=(self.slot_g, None), outs=(self.packed, None),
                                       bits=(self.bits_g, None), offs=(self.word_off, None))
            if self.world > 1:
                self.gathered = gather_streams(self.packed, self.word_off[-1:], self.world, self.rank)
        self.k += 1

    def collect(self):
        """after the timed steps (collective): every rank's per-frame bit counts and a fingerprint of
        its input frames, on every rank"""
        per = (self.TOTAL + self.world - 1) // self.world
        b = [int(x) for x in self.pybic.as_u64(self.bits_g[:self.nplanes])] + [0] * (per - self.nplanes)
        self.allbits = allgather_i64(b, self.world, self.ctx.dev)
        self.sums = allgather_i64(checksum(self.planes[:self.nplanes]), self.world, self.ctx.dev)

    def kernel_bytes(self):
        plane_b = self.nplanes * self.rows * self.wpr * 8
        g = int(self.pybic.as_u64(self.bits_g[:self.nplanes]).astype(np.int64).sum()) // 8
        return {"med_count": plane_b, "golomb_bits": plane_b, "golomb_emit": plane_b + g,
                "encode_rows_golomb": plane_b + g}

    def check(self, oracle):
        """rank 0, after collect(): every one of the 64 frames' streams -- rank 0's own at its packed
        offsets at N = 1, the buffer rank 0 RECEIVED from the gather at N > 1 -- == the oracle's
        stream of that frame. Rank 0 regenerates the other ranks' frames from their seeds and
        checks them against the fingerprints those ranks sent."""
        if self.world == 1:
            W = self.pybic.as_u64(self.packed)
            offs = [0, int(self.pybic.as_u64(self.word_off)[-1])]
        else:
            W = self.pybic.as_u64(self.gathered[0])
            offs = self.gathered[1]
        ok = True
        nframes = 0
        for r in range(self.world):
            n = len(self.share(r))
            if n == 0:
                ok &= offs[r + 1] == offs[r]
                continue
            fr = self.planes if r == self.rank else self.frames_of(r)
            ok &= checksum(fr[:n]) == self.sums[r]
            P = self.pybic.as_u64(fr[:n])
            exp = oracle.encode_planes_par(P, self.cols, 1, coders=(0,))
            o = offs[r]
            for k in range(n):
                eb, est = exp[(k, 0)]
                nw = (eb + 63) // 64
                ok &= int(self.allbits[r][k]) == eb and W[o:o + nw].tobytes() == est.tobytes()
                o += nw
                nframes += 1
            ok &= o == offs[r + 1]
        return bool(ok and nframes == self.TOTAL)


class C5(C3):
    """8192x8192 plane, 32x32 tiles (compress7 R = 0 path): weights, mode, Golomb over tiles. On N
    GPUs the plane is split into bands of tile rows (strong scaling); the one adaptive coder over the
    tile sequence is continued across ranks by exchanging its state and bit offsets
    (pybic.parallel.sharded_golomb) and the stream is reassembled on rank 0."""

    def __init__(self, ctx, args, rank, world=1):
        import pybic
        t = ctx.torch
        self.ctx, self.pybic, self.rank, self.world = ctx, pybic, rank, world
        self.rows = args.rows or 8192
        self.cols = args.cols or 8192
        self.W = 32
        self.nplanes = 1
        self.wpr = (self.cols + 63) // 64
        self.band_rows = self.band(rank)
        self.planes = self.band_plane(rank)
        self.lt = pybic.lentab(self.W)
        self.res = None
        self.own_bits = 0
        self.merged = None
        self.k = 0
        self.pixels = self.band_rows * self.cols
        self.bits_e = ctx.torch.zeros(1, dtype=t.int64, device=ctx.dev)
        self.workload = (f"c5: {self.rows}x{self.cols} plane, 32x32 tiles, per-tile med/mode + Golomb over weights"
                         + (f", tile-row bands over {world} GPUs" if world > 1 else ""))

    def band(self, r):
        ny = self.rows // self.W
        return ((r + 1) * ny // self.world - r * ny // self.world) * self.W

    def band_plane(self, r):
        """rank r's band of tile rows (seeded per rank on the device; rank 0 regenerates any rank's)"""
        t = self.ctx.torch
        g = t.Generator(device=self.ctx.dev)
        g.manual_seed(0x5EED0000 + r)
        return rand_words(t, (1, self.band(r), self.wpr), self.ctx.dev, g)

    def collect(self):
        self.sums = allgather_i64(checksum(self.planes), self.world, self.ctx.dev)

    def step(self):
        c = self.ctx
        self.res = c.patch_encode(self.planes[0], self.cols, self.W, self.lt, want_resid=True, bufs=self.res)
        if self.world > 1:
            from pybic.parallel import sharded_golomb
            wts = self.res["weights"]
            total = int(self.pybic.as_u64(self.res["stats"])[1])

            def enc(n0, a0, bit0):
                out, bits = c.golomb_encode_samples(wts, n0=n0, a0=a0, bit0=bit0)
                nb = int(self.pybic.as_u64(bits)[0])
                self.own_bits = nb
                return out, nb
            def lengths(n0, a0):
                return int(self.pybic.as_u64(c.golomb_lengths(wts, n0=n0, a0=a0))[0])
            self.merged, self.merged_bits = sharded_golomb(enc, wts.numel(), total, c.dev, lengths=lengths)
        self.k += 1

    def out_bytes(self):
        if self.world > 1:
            return self.own_bits / 8.0
        return int(self.pybic.as_u64(self.res["stats"])[0]) / 8.0

    def kernel_bytes(self):
        return {"tiles": 2 * self.band_rows * self.wpr * 8}

    def check(self, oracle):
        """N = 1: the plane's stream, bit count and L == the oracle's. N > 1 (rank 0, after
        collect()): the MERGED stream rank 0 assembled from every band (one adaptive coder continued
        across the ranks) == the oracle's stream of the whole plane; rank 0 regenerates the other
        bands from their seeds and checks them against the fingerprints those ranks sent."""
        if self.world == 1:
            P = self.pybic.as_u64(self.planes[0])
            exp = oracle.patch_encode(P, self.cols, self.W, self.lt, want_stream=True)
            st = self.pybic.as_u64(self.res["stats"])
            return (int(st[0]) == exp["bits"] and int(st[2]) == exp["L"] and
                    self.pybic.stream_bytes(self.res["stream"], exp["bits"]) == exp["stream"].tobytes())
        bands = []
        ok = True
        for r in range(self.world):
            b = self.planes if r == self.rank else self.band_plane(r)
            ok &= checksum(b) == self.sums[r]
            bands.append(self.pybic.as_u64(b[0]))
        P = np.ascontiguousarray(np.concatenate(bands, axis=0))
        exp = oracle.patch_encode(P, self.cols, self.W, self.lt, want_stream=True)
        ok &= self.merged_bits == exp["bits"]
        ok &= self.pybic.stream_bytes(self.merged, exp["bits"]) == exp["stream"].tobytes()
        return bool(ok)


class C1(C3):
    """compress_test.cpp's patch match search (configs[0]: 512x512 PBM, W = 5): for every tile the
    least-distance window of the causal region -- the reference's dominant cost (§8 f2). Not part
    of the default bench; value = image pixels per second."""

    def __init__(self, ctx, args, rank):
        import pybic
        t = ctx.torch
        self.ctx, self.pybic = ctx, pybic
        self.rows = args.rows or 512
        self.cols = args.cols or 512
        self.W = 5
        self.nplanes = 1
        self.wpr = (self.cols + 63) // 64
        g = t.Generator(device=ctx.dev)
        g.manual_seed(0x5EED0000 + rank)
        self.planes = rand_words(t, (1, self.rows, self.wpr), ctx.dev, g)
        self.res = None
        self.k = 0
        self.pixels = self.rows * self.cols
        self.bits_e = ctx.torch.zeros(1, dtype=t.int64, device=ctx.dev)
        self.workload = f"c1: {self.rows}x{self.cols} plane, compress_test patch search, W = {self.W}"

    def step(self):
        self.res = self.ctx.patch_search(self.planes[0], self.cols, self.W)
        self.k += 1

    def out_bytes(self):
        return 0.0

    def kernel_bytes(self):
        return {}

    def candidates(self, rows):
        """windows the search visits for the tiles of the first `rows` rows (its work measure)"""
        W, cols, n = self.W, self.cols, 0
        for ti in range((rows + W - 1) // W):
            i0 = ti * W
            rows1 = i0 - W + 1 if i0 >= W else 0
            for tj in range((cols + W - 1) // W):
                j0 = tj * W
                n += rows1 * cols + ((i0 - rows1 + 1) * (j0 - W + 1) if j0 >= W else 0)
        return n

    def check(self, oracle):
        """the tiles of the first 60 rows depend on nothing below row 64: compare those"""
        sub = 60
        P = self.pybic.as_u64(self.planes[0])[:sub + self.W]
        exp = oracle.patch_search(P, self.cols, self.W)
        nx = (self.cols + self.W - 1) // self.W
        nt = (sub // self.W) * nx
        return all((g.cpu().numpy().view(np.uint32)[:nt] == e[:nt]).all() for g, e in zip(self.res, exp))

    def cpu_time(self, rows):
        """the search loop on the first `rows` rows, extrapolated to the whole image by the exact count of
        visited windows: the reference's own loop over its binmat.cpp objects (ref_patch_search, kind
        "reference") where oracle/_ref is built (this container), else the oracle's restatement of it
        (kind "port": on the GPU box, where .gpurunignore keeps oracle/_ref out)"""
        from oracle_lib import Oracle, Ref, have_ref
        P = np.ascontiguousarray(self.pybic.as_u64(self.planes[0])[:rows])
        impl, kind = (Ref(), "reference") if have_ref() else (Oracle(), "port")
        t0 = time.perf_counter()
        impl.patch_search(P, self.cols, self.W)
        dt = time.perf_counter() - t0
        return dt * self.candidates(self.rows) / max(1, self.candidates(rows)), dt, kind


class C1M(C1):
    """compress7_test.cpp's whole tile loop with its default search window (W = 16, T = 0,
    R = 128) on configs[0]'s 512x512 plane: causal match search over the residual image, modes,
    write-back, the two Golomb coders (§8 f2). The input is a synthetic text-like page (glyphs of a
    small random alphabet), the kind of image the match search is for; value = pixels per second."""

    def __init__(self, ctx, args, rank):
        import pybic
        from oracle_lib import text_plane  # input generator only (numpy); not the checker
        self.ctx, self.pybic = ctx, pybic
        self.rows = args.rows or 512
        self.cols = args.cols or 512
        self.W, self.T, self.R = 16, 0, 128
        self.nplanes = 1
        self.wpr = (self.cols + 63) // 64
        self.host = text_plane(0x5EED + rank, self.rows, self.cols)
        self.planes = ctx.to_dev(self.host)[None]
        self.enuml = pybic.enum_table(self.W)
        self.resid = ctx.empty_i64(self.rows, self.wpr)
        self.res = None
        self.k = 0
        self.pixels = self.rows * self.cols
        self.workload = (f"c1m: {self.rows}x{self.cols} text-like plane, compress7_test tile loop, "
                         f"W = {self.W}, T = {self.T}, R = {self.R}")

    def step(self):
        self.res = self.ctx.match_encode(self.planes[0], self.cols, self.W, self.T, self.R, self.enuml,
                                         resid=self.resid)
        self.k += 1

    def out_bytes(self):
        st = self.pybic.as_u64(self.res["stats"])
        return (int(st[1]) + int(st[2]) + int(st[3])) / 8.0

    def check(self, oracle):
        exp = oracle.match_encode(self.host, self.cols, self.W, self.T, self.R, self.enuml)
        st = [int(x) for x in self.pybic.as_u64(self.res["stats"])]
        return (st == [exp["matches"], exp["bits_match"], exp["bits_nomatch"], exp["L"]] and
                bool((self.pybic.as_u64(self.resid) == exp["residual"]).all()))

    def cpu_time(self, rows):
        """the oracle's restatement of the driver's loop, whole image"""
        from oracle_lib import Oracle
        impl, kind = Oracle(), "port"
        t0 = time.perf_counter()
        if kind == "reference":
            impl.match_loop(self.host, self.cols, self.W, self.T, self.R, self.enuml)
        else:
            impl.match_encode(self.host, self.cols, self.W, self.T, self.R, self.enuml, want_stream=False)
        dt = time.perf_counter() - t0
        return dt, dt, kind


# ------------------------------------------------------------------------------------------
def cpu_baseline(wl, args):
    """The oracle's restatement of the reference's bit-serial med + GolombCoder + EGCoder (kind
    "port", the streams written) on a bounded sample of the same workload, OpenMP over independent
    planes, on this host's cores; plus the word-parallel CPU encoder as `strong`."""
    from oracle_lib import Oracle
    if isinstance(wl, C1M):
        est, dt, kind = wl.cpu_time(wl.rows)
        return {"value": wl.pixels / est / 1e6, "unit": "MPix/s", "cores": 1, "kind": kind,
                "sample": f"the whole {wl.rows}x{wl.cols} loop once ({dt:.1f} s, single thread: the loop is "
                          f"serial)"}
    if isinstance(wl, C1):
        sample_rows = min(wl.rows, 120)
        est, dt, kind = wl.cpu_time(sample_rows)
        return {"value": wl.pixels / est / 1e6, "unit": "MPix/s", "cores": 1, "kind": kind,
                "sample": f"search of the tiles in the first {sample_rows} rows ({dt:.1f} s, single thread: the "
                          f"reference loop is serial), extrapolated to the {wl.rows}x{wl.cols} image by the count "
                          f"of windows visited ({est:.1f} s)"}
    rows = min(args.cpu_rows, wl.rows)
    planes = np.ascontiguousarray(wl.host_planes(rows)) if hasattr(wl, "host_planes") else None
    if planes is None:
        return None
    nplanes = planes.shape[0]
    threads = max(1, min(nplanes, int(os.environ.get("OMP_NUM_THREADS", "8") or 8)))
    do_eg = 1 if type(wl) in (C3, C3Planes, C3File) else 0
    predict = 0 if isinstance(wl, C2) else 1
    reps, dt, used = 0, 0.0, 0
    # the restatement (BASELINE.md's plan): bit-serial med, serial GolombCoder / EGCoder, the streams
    # written; OpenMP over planes. (The reference's own objects stay an in-container cross-check:
    # oracle/_ref does not travel to the GPU box.)
    import ctypes as C
    o = Oracle()
    while reps == 0 or (dt < args.cpu_seconds and reps < 32):
        used_c = C.c_int(0)
        t0 = time.perf_counter()
        o.lib.bo_baseline_planes(planes.ctypes.data_as(C.POINTER(C.c_uint64)), nplanes, rows, wl.cols,
                                 planes.shape[-1], predict, do_eg, C.byref(used_c))
        t, used, kind = time.perf_counter() - t0, used_c.value, "port"
        dt += t
        reps += 1
    px = reps * nplanes * rows * wl.cols
    what = 'med+Golomb+EG' if do_eg else ('med+Golomb' if predict else 'Golomb')
    host = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    out = {"value": px / dt / 1e6, "unit": "MPix/s", "cores": int(min(used, nplanes)), "kind": kind,
           "sample": f"{nplanes} planes x {rows} rows x {wl.cols} cols (first {rows} rows of the bench input), "
                     f"{what}, the streams written bit by bit (bo_encode_plane, the oracle's restatement of "
                     f"pred.cpp / GolombCoder.cpp / eg.cpp), "
                     f"OpenMP over planes (one coder per plane: at most {nplanes} threads), {reps} repetitions, "
                     f"{dt:.2f} s",
           "host": host}
    # the strong CPU line (BASELINE.md plan): a word-parallel restatement (oracle/cpu_fast.c) writing the
    # same streams as the GPU, OpenMP over planes, on the same sample
    o = Oracle()
    reps2, dt2, used2 = 0, 0.0, 0
    while reps2 == 0 or (dt2 < args.cpu_seconds / 2 and reps2 < 64):
        t0 = time.perf_counter()
        *_, used2 = o.fast_encode(planes, wl.cols, predict, do_eg=do_eg)
        dt2 += time.perf_counter() - t0
        reps2 += 1
    out["strong"] = {"value": reps2 * nplanes * rows * wl.cols / dt2 / 1e6, "unit": "MPix/s", "cores": used2,
                     "kind": "port", "sample": f"the same sample, {what} streams written (word-parallel med, clz runs, "
                                               f"64-bit bit writer), {reps2} repetitions, {dt2:.2f} s"}
    return out


def main():
    args = parse()
    rc = spawn_ranks(args)  # before torch / HIP are touched in this process
    if rc is not None:
        sys.exit(rc)
    import torch
    world, rank, local = dist_setup(args)
    import pybic
    ctx = pybic.Context(local)
    ctx.set_encoder(args.encoder)
    if args.one_stream:
        ctx.set_one_stream(True)
    if args.workload == "c3" and args.shard == "planes":
        wl = C3Planes(ctx, args, rank, world)
    elif args.workload == "c3":
        wl = C3(ctx, args, rank)
    elif args.workload == "c3f":
        wl = C3File(ctx, args, rank)
    elif args.workload == "c2":
        wl = C2(ctx, args, rank)
    elif args.workload == "c4":
        wl = C4(ctx, args, rank, world)
    elif args.workload == "c1":
        wl = C1(ctx, args, rank)
    elif args.workload == "c1m":
        wl = C1M(ctx, args, rank)
    else:
        wl = C5(ctx, args, rank, world)
    dev = ctx.dev
    for _ in range(args.warmup):
        wl.step()
    ctx.sync()
    # per-kernel breakdown (every launch bracketed by HIP events) on untimed steps: it names the
    # dominant kernel. Event pairs drain the pipeline between launches (≈45 µs of a 0.5 ms C3
    # step with all of them), so the timed region below brackets only the dominant kernel.
    ctx.prof_enable(True)
    ctx.prof_only(None)
    for _ in range(max(args.warmup, 2)):
        wl.step()
    ctx.sync()
    prof_all = ctx.prof_collect()
    kb = wl.kernel_bytes()
    timed = {k: v for k, v in prof_all.items() if k in kb}
    dom = max(timed, key=lambda k: timed[k][1]) if timed else None
    ctx.prof_only(dom)
    if not dom:
        ctx.prof_enable(False)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step()
    barrier(world)
    dt = time.perf_counter() - t0
    ctx.sync()
    prof = ctx.prof_collect()
    ctx.prof_enable(False)
    ctx.prof_only(None)
    dt_max = max_over_ranks(dt, world, dev)
    pixels_all = sum_over_ranks(float(wl.pixels), world, dev) * args.steps
    out_all = sum_over_ranks(wl.out_bytes(), world, dev) * args.steps
    value = pixels_all / dt_max / 1e6
    # dominant kernel and its roofline (algorithmic bytes / its average launch time, measured with
    # HIP events inside the timed region)
    kb = wl.kernel_bytes()
    roof = None
    per_kernel = {k: {"launches": n, "avg_us": 1e3 * ms / max(n, 1)} for k, (n, ms) in prof_all.items()}
    if dom and dom in prof:
        timed = {dom: prof[dom]}
        n, ms = timed[dom]
        avg_s = ms / 1e3 / n
        ach = kb[dom] / avg_s / 1e9
        traffic, tnote = load_pmc(args.workload, dom)
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tnote, "kernel": dom,
                "algorithmic_bytes_per_launch": kb[dom], "avg_launch_us": round(avg_s * 1e6, 2)}
        st = per_kernel.get(dom + "_stage")
        if st:  # the staged encoder's emission: the main kernel timed alone, the whole stage beside it
            roof["stage_avg_us"] = round(st["avg_us"], 2)
            roof["note"] = ("avg_launch_us: HIP events on the launch stream right around the main emission kernel "
                            "(k_emit_k01 / k_emit_known; k_emit_rest's ~1 % of the rows run beside it on a second "
                            "stream and their bytes are counted too); stage_avg_us: the whole stage, that second "
                            "stream's fork and join included (untimed profiled steps)")
    pred_pass = wl.predictor_pass(max(args.steps, 5)) if hasattr(wl, "predictor_pass") and type(wl) is C3 else None
    if pred_pass is not None and "bitplanes_count" in per_kernel:
        # the pass that runs inside the step: bic_encode_gray's count pass (k_gray_strips: gray -> planes,
        # med residual, per-strip run statistics), gray read + planes written, alternating images
        us = per_kernel["bitplanes_count"]["avg_us"]
        b = kb["bitplanes_count"]
        pred_pass["in_step"] = {"kernel": "bitplanes_count (k_gray_strips)", "algorithmic_bytes_per_launch": b,
                                "achieved": round(b / us / 1e3, 1), "frac": round(b / us / 1e3 / HBM_PEAK_GBS, 4),
                                "avg_launch_us": round(us, 2)}
    if hasattr(wl, "collect"):
        wl.collect()
    ok = None
    cpu = None
    if rank == 0 and not args.no_check:
        from oracle_lib import Oracle
        ok = bool(wl.check(Oracle()))
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(wl, args)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "MPix/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt_max / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong" if args.workload in ("c4", "c5") or isinstance(wl, C3Planes) else "weak", "vs_baseline": None, "dtype": "u64",
            "data": ("synthetic text-like page (seeded glyph alphabet), device-resident" if args.workload == "c1m"
                     else "synthetic (seeded uniform bytes / Bernoulli(0.5) words, device-resident)"),
            "config": {"workload": wl.workload, "rows": wl.rows, "cols": wl.cols, "planes_per_gpu": wl.nplanes,
                       "parallelism": f"dp{world} (planes of one image sharded, streams gathered to rank 0)"
                       if isinstance(wl, C3Planes) else {"c4": f"dp{world} (64 frames sharded)",
                                       "c5": f"dp{world} (tile-row bands, coder state exchanged)"}.get(
                                           args.workload, f"dp{world} (independent images per GPU)")},
            "mb_per_s_out": round(out_all / dt_max / 1e6, 1),
            "gray_mpix_per_s": round(value / 8, 1) if args.workload == "c3" else None,
            "roofline": roof, "predictor_pass": pred_pass, "kernels": per_kernel,
            "kernels_note": "all launches event-bracketed on untimed steps; the timed region brackets only roofline.kernel",
            "bit_exact_check": ok, "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    ctx.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
