"""Device-resident stripes: plans over shards already in HBM.

A *stripe* is one object's n = k+m shards. `StripeBatch` lays a batch of stripes out
in HBM: by default in one allocation, `[batch][n][pitch]` bytes (pitch = S rounded up to
256 B so every shard starts 16-B aligned for the vector kernel), the layout the GPU
tests use; the benchmark's `planar` layout keeps the data shards and the parity in two
regions, and the Split layouts reproduce upstream's (see the class). `Plan` wraps rs_plan_create/rs_plan_launch: the
coefficient tables and shard-pointer tables are uploaded once, and each launch only
enqueues kernels on the given stream (capturable in a HIP graph).

PyTorch is only the allocator and stream provider here; the arithmetic is the HIP
kernels in libcallfs_rs.so.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch

from . import _native as N


def pitch_for(S: int) -> int:
    return (S + 255) // 256 * 256


def _aligned_empty(shape, align: int, device) -> torch.Tensor:
    """An uninitialised uint8 tensor of `shape` whose first byte is `align`-aligned."""
    n = 1
    for d in shape:
        n *= d
    raw = torch.empty(n + align, dtype=torch.uint8, device=device)
    off = -raw.data_ptr() % align
    return raw[off:off + n].view(shape)


class StripeBatch:
    """`batch` stripes of RS(k, m) with shard size S, resident on `device`.

    layout "pitch" (default): shards at a 256-B pitch, every shard 16-B aligned.
    layout "split": upstream `Split`'s layout of contiguous objects (codec.go:31) when the
    body's capacity holds all n shards: pitch = S, object b's shard i at b*n*S + i*S, so
    at odd S every shard but the first sits at its own byte offset (the realigning
    kernel's case).
    layout "planar": the pitch layout's 256-B shard pitch, but the k data shards of every
    stripe in one region ([batch][k][pitch]) and the m parity shards in another
    ([batch][m][pitch]), so no stripe's parity sits between two stripes' data.
    layout "shardmajor": the 256-B pitch with all stripes' shard i in one region
    ([n][batch][pitch]).
    layout "readall": upstream `Split` of a body whose capacity holds the k data shards
    but not the parity, which is what CallFS passes it: io.ReadAll's body
    (post_file_enhanced.go:127) grows by append, so cap/len stays below n/k for every
    profile with m/k > 1/4. The data shards are slices of the body at pitch S (body
    bases `BODY_ALIGN`-aligned, as the Go heap's large objects are page-aligned); the m
    parity shards come from reedsolomon's AllocAligned: 64-B aligned, each at a pitch of
    S rounded up to 64 B (klauspost/reedsolomon v1.13.3 reedsolomon.go Split,
    galois.go AllocAligned)."""

    BODY_ALIGN = 8192

    def __init__(self, k: int, m: int, S: int, batch: int, device: torch.device,
                 layout: str = "pitch", pitch: Optional[int] = None):
        """pitch: shard pitch in bytes for the 'pitch', 'planar' and 'shardmajor' layouts
        (a multiple of 16, at least S; default pitch_for(S), the library's own rule)."""
        if layout not in ("pitch", "split", "readall", "planar", "shardmajor"):
            raise ValueError(f"layout {layout!r}")
        if pitch is not None and (layout in ("split", "readall") or pitch < S or pitch % 16):
            raise ValueError(f"pitch {pitch} for layout {layout!r}, S = {S}")
        self.k, self.m, self.S, self.batch = k, m, S, batch
        self.n = k + m
        self.layout = layout
        self.device = torch.device(device)
        if layout in ("readall", "planar"):
            # data shard i of stripe b at body + b*body_pitch + i*pitch, parity j at
            # par + (b*m + j)*par_pitch
            if layout == "readall":
                self.pitch = S
                self.body_pitch = -(-k * S // self.BODY_ALIGN) * self.BODY_ALIGN
                self.par_pitch = -(-S // 64) * 64
            else:
                self.pitch = self.par_pitch = pitch or pitch_for(S)
                self.body_pitch = k * self.pitch
            self.body = _aligned_empty((batch, self.body_pitch), self.BODY_ALIGN, self.device)
            self.par = _aligned_empty((batch, m, self.par_pitch), 256, self.device)
            self.buf = None
            return
        self.pitch = S if layout == "split" else (pitch or pitch_for(S))
        if layout == "shardmajor":
            sm = torch.empty((self.n, batch, self.pitch), dtype=torch.uint8, device=self.device)
            self.buf = sm.permute(1, 0, 2)  # [batch][n][pitch] view of [n][batch][pitch]
            return
        self.buf = torch.empty((batch, self.n, self.pitch), dtype=torch.uint8, device=self.device)

    def shard(self, b: int, i: int) -> torch.Tensor:
        if self.buf is None:
            if i < self.k:
                return self.body[b, i * self.pitch:i * self.pitch + self.S]
            return self.par[b, i - self.k, : self.S]
        return self.buf[b, i, : self.S]

    def data(self) -> torch.Tensor:
        if self.buf is None:
            return self.body[:, : self.k * self.pitch].view(self.batch, self.k, self.pitch)[:, :, : self.S]
        return self.buf[:, : self.k, : self.S]

    def parity(self) -> torch.Tensor:
        if self.buf is None:
            return self.par[:, :, : self.S]
        return self.buf[:, self.k:, : self.S]

    def gather(self, stripes: Optional[int] = None) -> torch.Tensor:
        """A [stripes][n][S] copy of the first `stripes` stripes' shards (all by default)."""
        ns = self.batch if stripes is None else stripes
        if self.buf is None:
            return torch.cat([self.data()[:ns], self.parity()[:ns]], dim=1)
        return self.buf[:ns, :, : self.S].clone()

    def zero_shard(self, i: int) -> None:
        """Zero shard i of every stripe."""
        if self.buf is None:
            (self.data()[:, i] if i < self.k else self.parity()[:, i - self.k]).zero_()
        else:
            self.buf[:, i, : self.S].zero_()

    def pointers(self) -> list:
        if self.buf is None:
            body, par = self.body.data_ptr(), self.par.data_ptr()
            return [body + b * self.body_pitch + i * self.pitch if i < self.k
                    else par + (b * self.m + i - self.k) * self.par_pitch
                    for b in range(self.batch) for i in range(self.n)]
        base = self.buf.data_ptr()
        sb_, si_ = self.buf.stride(0), self.buf.stride(1)
        return [base + b * sb_ + i * si_ for b in range(self.batch) for i in range(self.n)]

    def fill_random(self, seed: int) -> None:
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        for t in ((self.buf,) if self.buf is not None else (self.body, self.par)):
            t.random_(0, 256, generator=g)


class Plan:
    """rs_plan over explicit device shard pointers (batch*n of them, stripe-major).

    present=None is an encode plan (data present, parity missing); otherwise the
    missing shards are reconstructed from the first k present ones and the remaining
    present parity is re-verified (codec.go:55,59).
    """

    def __init__(self, k: int, m: int, S: int, batch: int, pointers: Sequence[int],
                 present: Optional[Sequence[bool]] = None, device: int = 0,
                 context: Optional[N.Context] = None):
        self.ctx = context or N.default_context()
        n = k + m
        if len(pointers) != batch * n:
            raise ValueError("need batch*(k+m) shard pointers")
        self.k, self.m, self.S, self.batch, self.device = k, m, S, batch, device
        ptrs = (ctypes.c_void_p * len(pointers))(*pointers)
        pres = None
        if present is not None:
            if len(present) != n:
                raise ValueError("present needs k+m flags")
            pres = (ctypes.c_uint8 * n)(*[1 if p else 0 for p in present])
        h = ctypes.c_void_p()
        N.check(N.lib.rs_plan_create(self.ctx.handle, device, k, m, S, batch, pres, ptrs,
                                     ctypes.byref(h)), "rs_plan_create")
        self.handle = h

    @classmethod
    def for_batch(cls, sb: StripeBatch, present=None, context=None) -> "Plan":
        dev = sb.device.index if sb.device.index is not None else 0
        return cls(sb.k, sb.m, sb.S, sb.batch, sb.pointers(), present, dev, context)

    @property
    def bytes(self) -> int:
        """Algorithmic HBM bytes one launch moves."""
        return int(N.lib.rs_plan_bytes(self.handle))

    def launch(self, stream: Optional[torch.cuda.Stream] = None, events=None) -> None:
        """rs_plan_launch; events = (start, stop) torch.cuda.Event pair (timing enabled,
        recorded at least once so the HIP events exist): rs_plan_launch_timed, the
        first kernel dispatch records start when it starts and the last records stop when
        it ends, so start.elapsed_time(stop) is the kernels' own time."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if events is None:
            N.check(N.lib.rs_plan_launch(self.handle, ctypes.c_void_p(s.cuda_stream)),
                    "rs_plan_launch")
            return
        h = [ctypes.c_void_p(e.cuda_event) for e in events]
        if not all(x.value for x in h):
            raise ValueError("record each event once before timing launches with it")
        N.check(N.lib.rs_plan_launch_timed(self.handle, ctypes.c_void_p(s.cuda_stream), *h),
                "rs_plan_launch_timed")

    CEILINGS = {"nolookup": 0, "read": 1, "write": 2, "write64": 3, "write128": 4,
                "write256": 5, "read64": 6, "read128": 7, "read256": 8}

    def launch_ceiling(self, mode: str = "read",
                       stream: Optional[torch.cuda.Stream] = None, events=None) -> None:
        """rs_plan_launch_ceiling (measurement only): this plan's read / write streams
        alone, same grid and tile order ("write" leaves junk in the written shards). The
        A/B build (CALLFS_RS_LIB) adds "nolookup" (the kernel's no-lookup form) and the
        aligned-window probes; the product refuses them (RS_E_ARG). events: as for launch()."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if events is None:
            N.check(N.lib.rs_plan_launch_ceiling(self.handle, ctypes.c_void_p(s.cuda_stream),
                                                 self.CEILINGS[mode]), "rs_plan_launch_ceiling")
            return
        h = [ctypes.c_void_p(e.cuda_event) for e in events]
        if not all(x.value for x in h):
            raise ValueError("record each event once before timing launches with it")
        N.check(N.lib.rs_plan_launch_ceiling_timed(self.handle, ctypes.c_void_p(s.cuda_stream),
                                                   self.CEILINGS[mode], *h),
                "rs_plan_launch_ceiling_timed")

    # tile orders (RS_ORDER_*); on misaligned shards 0..6 name the plain kernel with
    # unaligned accesses and "realign*" the kernel that aligns loads and stores
    ORDER_NAMES = {-1: "none", 0: "consecutive", 1: "g8", 2: "g2", 3: "q8", 4: "q16", 5: "x8",
                   6: "x32", 32: "realign", 37: "realign-x8", 38: "realign-x32",
                   64: "wix", 65: "wix-g8", 66: "wix-g2", 67: "wix-q8", 68: "wix-q16",
                   69: "wix-x8", 70: "wix-x32", 96: "tri", 98: "tri-g2", 99: "tri-q8",
                   100: "tri-q16", 101: "tri-x8", 102: "tri-x32", 128: "realign-tri", 133: "realign-tri-x8",
                   134: "realign-tri-x32", 160: "realign64", 165: "realign64-x8",
                   166: "realign64-x32", 192: "dma", 194: "dma-g2", 195: "dma-q8",
                   198: "dma-x32", 224: "tridb-g4", 225: "tridb-g8", 256: "bs", 257: "bs-g8",
                   258: "bs-g2", 259: "bs-q8", 260: "bs-q16", 261: "bs-x8", 262: "bs-x32"}

    def tune(self, reps: int = 5, stream: Optional[torch.cuda.Stream] = None) -> list:
        """rs_plan_tune: time each launch group in every tile order its kernel offers
        and keep the fastest for later launches (synchronous; outputs recomputed to the
        same bytes). Returns the chosen order name per launch group."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        n = int(N.lib.rs_plan_groups(self.handle))  # one entry per launch group
        orders = (ctypes.c_int * n)()
        N.check(N.lib.rs_plan_tune(self.handle, ctypes.c_void_p(s.cuda_stream), reps, orders, n),
                "rs_plan_tune")
        return [self.ORDER_NAMES.get(orders[i], str(orders[i])) for i in range(n)]

    def set_orders(self, names: Sequence[str]) -> None:
        """rs_plan_set_orders: pin launch group i to tile order names[i] ("none" = the
        rule). An order the group's kernel does not offer raises NativeError (RS_E_ARG)
        and leaves the plan unchanged."""
        codes = {v: k for k, v in self.ORDER_NAMES.items()}
        arr = (ctypes.c_int * len(names))(*[codes[nm] for nm in names])
        N.check(N.lib.rs_plan_set_orders(self.handle, arr, len(names)), "rs_plan_set_orders")

    def forms(self) -> list:
        """rs_plan_forms: the kernel form (order name) each launch group of the next launch
        runs: the pinned or tuned order, else the rule's ("bs-*" once the rule's bit-sliced
        kernel is compiled)."""
        n = int(N.lib.rs_plan_groups(self.handle))
        out = (ctypes.c_int * max(n, 1))()
        got = N.lib.rs_plan_forms(self.handle, out, n)
        if got < 0:
            N.check(got, "rs_plan_forms")
        return [self.ORDER_NAMES.get(out[i], str(out[i])) for i in range(n)]

    def corrupt(self, stream: Optional[torch.cuda.Stream] = None) -> bool:
        """Synchronises the stream; True when a Verify row mismatched (then clears)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        c = ctypes.c_int(0)
        N.check(N.lib.rs_plan_status(self.handle, ctypes.c_void_p(s.cuda_stream),
                                     ctypes.byref(c)), "rs_plan_status")
        return bool(c.value)

    def corrupt_stripes(self, stream: Optional[torch.cuda.Stream] = None) -> list:
        """Synchronises the stream; indices of the stripes whose Verify rows mismatched
        since the last status call (then clears)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        flags = (ctypes.c_int * self.batch)()
        N.check(N.lib.rs_plan_stripe_status(self.handle, ctypes.c_void_p(s.cuda_stream), flags),
                "rs_plan_stripe_status")
        return [b for b in range(self.batch) if flags[b]]

    def close(self) -> None:
        if getattr(self, "handle", None):
            N.lib.rs_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HashPlan:
    """Batched SHA-256 (erasure.ShardChecksum, codec.go:81-84) of device-resident
    messages: rs_sha256_plan_* over `pointers`/`lengths` (device addresses, bytes)."""

    def __init__(self, pointers: Sequence[int], lengths: Sequence[int], device: int = 0,
                 context: Optional[N.Context] = None):
        self.ctx = context or N.default_context()
        if len(pointers) != len(lengths):
            raise ValueError("pointers/lengths length mismatch")
        self.count = len(pointers)
        self.device = device
        ptrs = (ctypes.c_void_p * max(1, self.count))(*pointers)
        lens = (ctypes.c_uint64 * max(1, self.count))(*lengths)
        h = ctypes.c_void_p()
        N.check(N.lib.rs_sha256_plan_create(self.ctx.handle, device, ptrs, lens, self.count,
                                            ctypes.byref(h)), "rs_sha256_plan_create")
        self.handle = h

    def launch(self, digests: torch.Tensor, stream: Optional[torch.cuda.Stream] = None) -> None:
        """digests: uint8 CUDA tensor of at least 32*count bytes (4-B aligned)."""
        if digests.dtype != torch.uint8 or digests.numel() < 32 * self.count:
            raise ValueError("need a uint8 tensor of 32*count bytes")
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        N.check(N.lib.rs_sha256_plan_launch(self.handle, ctypes.c_void_p(digests.data_ptr()),
                                            ctypes.c_void_p(s.cuda_stream)), "rs_sha256_plan_launch")

    def hexdigests(self) -> list:
        out = torch.empty(32 * max(1, self.count), dtype=torch.uint8,
                          device=torch.device("cuda", self.device))
        self.launch(out)
        raw = out.cpu().numpy().tobytes()
        return [raw[32 * i:32 * (i + 1)].hex() for i in range(self.count)]

    def close(self) -> None:
        if getattr(self, "handle", None):
            N.lib.rs_sha256_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_checksums(sb: StripeBatch) -> list:
    """ShardChecksum of every shard of a device-resident batch: [stripe][shard] hex."""
    dev = sb.device.index if sb.device.index is not None else 0
    hp = HashPlan(sb.pointers(), [sb.S] * (sb.batch * sb.n), dev)
    flat = hp.hexdigests()
    hp.close()
    return [flat[b * sb.n:(b + 1) * sb.n] for b in range(sb.batch)]
