#!/usr/bin/env python3
"""bench.py — device-resident RS(10,4) encode+decode on MI355X (BASELINE.json metric).

Workload (N=1 line; BASELINE.json metric "GiB/s device-resident RS encode+decode
(k=10,m=4, 1 MiB shards)"): every GPU holds `--stripes` stripes of RS(k, m) with S-byte
shards in HBM ([stripe][shard][pitch] layout). One *step* is one pass of the hot path
over that batch:
  1. encode  — parity of every stripe from its k data shards     (codec.go:36)
  2. decode  — reconstruct the erased shards (--erase, default {0,1,2,3}, the
               worst case of configs[2]) from the first k present ones and
               re-verify any remaining present parity               (codec.go:55,59)
value = user bytes through both ops (2 * stripes * k * S per GPU per step) summed over
all ranks / the max-over-ranks wall time of the timed steps, in GiB/s.

Layout (since round 4; rounds 1-3 kept each stripe's n shards in one block, `--layout
pitch`): the data shards in one HBM region and the parity in another (`planar`), erased
shards rebuilt into fresh buffers. At the metric's 1 MiB shards this is how upstream Split
lays out a 10 MiB io.ReadAll body whose capacity ends at its length (data at a 1 MiB pitch
in the body, parity in AllocAligned buffers), and the buffers upstream Reconstruct
allocates; `layout_ab` in the line times the same kernels in the same process in the old
layout (`pitch`) and in upstream Split of an io.ReadAll body per object (`readall`, decode
into fresh buffers).

Multi-GPU: one process per GPU (torch.distributed.run); stripes are independent, so
each rank encodes/decodes its own batch with no data-path collective ("weak"
scaling). The only cross-rank traffic is the gloo barrier and the max-reduce of the
timer.

roofline: the encode kernel's (rs_apply_lds for k >= 4) algorithmic bytes per launch
((k+m)*S per stripe) over its average HIP-event duration on the launch stream, against
8.0 TB/s HBM3E. The events are recorded by the kernel dispatches themselves
(rs_plan_launch_timed, hipExtLaunchKernel: start when the plan's first dispatch starts,
stop when its last ends), i.e. the kernel time rocprofv3's kernel trace reports; the
stream's gap between one launch and the next is in ms_per_step (and `launch_gap_ms`),
not in the per-kernel time.
cpu_baseline: rank 0 at N=1 only — the C port of the reference CPU algorithm
(oracle/rs_oracle.c orc_bench_codec: upstream GFNI/AVX2 kernels, one native loop,
stripe-parallel and byte-range threadings, the faster reported) over >= 2 GiB of the
same stripes copied to the host; the same leg checks the GPU parity and
reconstruction of those stripes bit-exactly against it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "GiB/s device-resident RS encode+decode (k=10,m=4, 1 MiB shards); % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
# host threads per GPU on the driver's boxes: a 1-GPU box grants 16 CPUs though
# sched_getaffinity / nproc list every CPU of the host
CPU_SHARE = 16


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=4)
    p.add_argument("--shard-bytes", type=int, default=1 << 20)
    p.add_argument("--stripes", type=int, default=None,
                   help="stripes per GPU (default 256; with --object-bytes: objects in total, "
                        "default as many as keep ~16 GiB of shards resident on one GPU)")
    p.add_argument("--object-bytes", type=int, default=0,
                   help="configs[3] mode: objects of this size (e.g. 1073741824) split by byte "
                        "columns across the ranks (strong scaling); --stripes objects in total")
    p.add_argument("--erase", default="0,1,2,3", help="erased shard indices for decode")
    p.add_argument("--layout", default="planar", choices=("planar", "pitch", "split", "readall"),
                   help="shard layout in HBM (device.StripeBatch): 'planar' (default since round "
                        "4: 256-B shard pitch, every stripe's data shards in one region and its "
                        "parity in another), 'pitch' (the same pitch, each stripe's n shards in one "
                        "block: rounds 1-3), or an upstream Split layout (--split-layout)")
    p.add_argument("--pitch", type=int, default=None,
                   help="shard pitch in bytes for --layout planar / pitch (a multiple of 16, "
                        ">= S; default: the library's planar_pitch rule, DESIGN.md §4)")
    p.add_argument("--decode-into", default="fresh", choices=("fresh", "inplace"),
                   help="with --layout planar or readall: rebuild the erased shards into a "
                        "region of their own ('fresh', as reedsolomon's Reconstruct allocates "
                        "missing shards) or into their slots of the batch ('inplace')")
    p.add_argument("--layout-ab", type=int, default=1,
                   help="1: with --layout planar, also time the same workload's kernels in the "
                        "'pitch' and 'readall' layouts in this process (tuned as well): "
                        "line['layout_ab']")
    p.add_argument("--split-layout", nargs="?", const="split", default=None,
                   choices=("split", "readall"),
                   help="upstream Split layout (codec.go:31) instead of the 256-B shard "
                        "pitch (configs[1]: --shard-bytes 6710887, misaligned shards at odd "
                        "S). 'split' (the bare flag): each object's n shards contiguous at "
                        "pitch = S, objects back to back (a body whose capacity holds all n "
                        "shards); 'readall': the data shards at pitch = S in page-aligned "
                        "bodies, the parity in reedsolomon's 64-B AllocAligned buffers (a "
                        "body from io.ReadAll, as CallFS passes it; device.StripeBatch)")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="CPU baseline time budget (0 disables)")
    p.add_argument("--cpu-working-set", type=int, default=2 << 30,
                   help="bytes of stripes the CPU baseline rotates through (>= 2 GiB: not "
                        "cache-resident)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU baseline threads (0: the visible cores, at most CPU_SHARE = 16, "
                        "the GPU box's CPU share per GPU)")
    p.add_argument("--tune", type=int, default=1,
                   help="1: rs_plan_tune each plan before the warmup (times every tile order "
                        "its kernel offers on this box and keeps the fastest; 0: the rule)")
    p.add_argument("--ceiling", type=int, default=1,
                   help="1: also time each plan's traffic ceilings in this process (its read "
                        "and write streams alone, and the kernel's no-lookup form; "
                        "roofline.copy_ceiling / roofline.nolookup)")
    p.add_argument("--traffic", default=os.path.join(HERE, "profiles", "hbm_traffic.json"),
                   help="PMC-measured HBM bytes per launch (rocprofv3 --pmc), if present")
    return p.parse_args(argv)


def cpu_quota_cores():
    """CPUs the process's cgroup grants (cgroup v2 cpu.max, else v1 cfs quota/period), or
    None when unlimited or unreadable: the GPU box's affinity mask lists every host CPU,
    but its cgroup may grant far fewer."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as fh:
                txt = fh.read().strip()
            if parse:
                q, per = parse(txt)
                return None if q == "max" else round(int(q) / int(per), 2)
            q = int(txt)
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                per = int(fh.read().strip())
            return None if q <= 0 else round(q / per, 2)
        except (OSError, ValueError):
            continue
    return None


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def cpu_baseline(sb, k, m, erase, seconds, ws_bytes, threads, all_threads=0, rebuilt=None):
    """Reference CPU path (port) timed natively on >= ws_bytes of the GPU's own stripes.

    oracle/rs_oracle.c orc_bench_codec runs upstream's per-object work -- Encode
    (codec.go:36), then Decode = Reconstruct from the first k present (codec.go:55) +
    Verify (codec.go:59) -- with the GFNI/AVX2 kernels of the port, in one native loop
    (no per-shard Python calls), in two threadings:
      stripe-parallel  each thread takes whole stripes (concurrent requests)
      byte-range       each op of each stripe split over all threads (codeSomeShardsP)
    `value` is the faster of the two. With all_threads > threads, modes["all-visible"]
    adds stripe-parallel at min(all_threads, sampled stripes) threads: every core the
    process may run on, beside the per-GPU share `value` is quoted at.
    Before timing, every sampled stripe is checked
    bit-exactly: CPU parity of the GPU's data == the GPU's parity, and the CPU
    reconstruction of the erased shards == the GPU's. With `rebuilt` (the decode writes
    into fresh buffers, [stripe][erased][pitch]) the host sample's erased shards are the
    GPU-rebuilt ones, so the CPU reconstruction is compared with the GPU's own output."""
    import numpy as np
    from oracle import cref

    S, n = sb.S, sb.n
    stripe_bytes = n * S
    ns = max(1, min(sb.batch, -(-ws_bytes // stripe_bytes)))
    host = sb.gather(ns).cpu().numpy()  # GPU-encoded + GPU-decoded stripes, [ns][n][S]
    if rebuilt is not None and erase:
        host[:, erase, :S] = rebuilt[:ns, :, :S].cpu().numpy()
    present = [i not in erase for i in range(k + m)]

    # bit-exact checks on all ns stripes
    bad, _, _ = cref.bench_codec(host, k, m, S, ops=cref.BENCH_VERIFY, nthreads=threads,
                                 seconds=0)
    if bad:
        raise SystemExit(f"GPU parity != CPU port on {bad} (stripe, parity row) pairs")
    if erase:
        keep = host[:, erase, :S].copy()
        host[:, erase, :S] = 0
        cref.bench_codec(host, k, m, S, present=present, ops=cref.BENCH_RECONSTRUCT,
                         nthreads=threads, seconds=0)
        if not np.array_equal(host[:, erase, :S], keep):
            raise SystemExit("GPU reconstruction != CPU port")
        del keep

    modes = {}
    for mode in ("stripe-parallel", "byte-range"):
        mism, el, passes = cref.bench_codec(host, k, m, S, present=present, nthreads=threads,
                                            seconds=seconds / 2, mode=mode)
        if mism:
            raise SystemExit(f"CPU verify mismatch in the {mode} timing loop")
        modes[mode] = round(2 * passes * ns * k * S / el / 2**30, 3)
    best = max(modes, key=modes.get)
    extra = {}
    if all_threads > threads:
        nt = min(all_threads, ns, 256)  # (orc_bench_codec's pool holds 256 threads)
        mism, el, passes = cref.bench_codec(host, k, m, S, present=present, nthreads=nt,
                                            seconds=seconds / 2, mode="stripe-parallel")
        if mism:
            raise SystemExit("CPU verify mismatch in the all-visible timing loop")
        extra = {"all-visible": round(2 * passes * ns * k * S / el / 2**30, 3)}
    out = {
        "value": modes[best],
        "unit": "GiB/s",
        "cores": threads,
        "threads": threads,
        "mode": best,
        "modes": modes,
        "kind": "port",
        "impl": (f"oracle/rs_oracle.c orc_bench_codec ({cref.simd_kind()}): upstream Encode, "
                 "then Reconstruct (first k present) + Verify, one native loop"),
        "working_set_bytes": ns * stripe_bytes,
        "sample": (f"{ns} stripes x RS({k},{m}) x {S} B shards ({ns * stripe_bytes / 2**30:.2f} GiB, "
                   f"rotated), encode + decode(erase {sorted(erase)}), ~{seconds / 2:.0f} s per "
                   "threading"),
        "parity_check": (f"GPU parity == CPU port of the GPU's data shards"
                         + (" (the GPU-rebuilt ones in the erased slots)" if rebuilt is not None
                            and erase else "")
                         + f", and the CPU reconstruction of the erased shards == the GPU's, "
                         f"bit-exact, on all {ns} sampled stripes"),
    }
    if extra:
        out["modes"].update(extra)
        out["all_visible_threads"] = min(all_threads, ns, 256)
        quota = cpu_quota_cores()
        out["cpu_quota_cores"] = quota
        out["all_visible_note"] = (
            f"stripe-parallel at {out['all_visible_threads']} threads (every CPU in the "
            f"affinity mask, capped by the {ns} sampled stripes): {extra['all-visible']} GiB/s "
            f"against {modes['stripe-parallel']} at {threads}; cgroup CPU quota "
            + (f"{quota} CPUs" if quota else "unlimited or unreadable")
            + ". More threads than the CPUs the box grants time-slice instead of running "
            "in parallel, so `value` stays the per-GPU share")
    return out


def _launch_ms(fn, stream, reps=20, warm_ms=30.0):
    """Mean ms per launch of fn(events) over `reps` launches, each timed by a pair of HIP
    events its kernel dispatches record (as the bench's own launches are), after >=
    warm_ms of untimed launches (a kernel timed right after a lighter or heavier one runs
    off its steady clock for milliseconds)."""
    with torch.cuda.stream(stream):
        t0 = time.perf_counter()
        while True:
            for _ in range(4):
                fn(None)
            torch.cuda.synchronize(stream.device)
            if (time.perf_counter() - t0) * 1e3 >= warm_ms:
                break
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        for a, b in ev:
            a.record(stream)
            b.record(stream)
        for pair in ev:
            fn(pair)
        torch.cuda.synchronize(stream.device)
    return sum(a.elapsed_time(b) for a, b in ev) / reps


def kernel_label(plan, k):
    """The kernel a plan's (first) launch group ran: the bit-sliced one generated for its
    coefficient block or the nibble-table / v_perm kernel."""
    form = plan.forms()[0]
    if form.startswith("bs"):
        return f"rs_bs (bit-sliced, generated for the plan's coefficients; {form})"
    return "rs_apply_lds" if k >= 4 else "rs_apply_vec"


def plan_ceilings(enc, dec, stream):
    """Same-process traffic ceilings of the two plans (rs_plan_launch_ceiling, DESIGN.md
    §6.1): each plan's read streams alone and write streams alone on the production grid
    and tile order -- their summed time is what the plan's bytes take when reads and writes
    each run at their own best rate, the achievable denominator -- and the production
    kernel's no-lookup form. Timed after the bench's timed steps; the plans are relaunched
    afterwards (decode first, then encode) so every shard holds its true bytes again."""
    from callfs_amd import _native as N
    out = {}
    for name, plan in (("decode", dec), ("encode", enc)):
        ms = {mode: _launch_ms(lambda evs: plan.launch_ceiling(mode, stream, events=evs), stream)
              for mode in ("read", "write")}
        try:  # the no-lookup form: A/B build of the library only (CALLFS_RS_LIB); the
            # product refuses the mode (RS_E_ARG: tools/callfs_rs_ab.h)
            ms["nolookup"] = _launch_ms(
                lambda evs: plan.launch_ceiling("nolookup", stream, events=evs), stream)
        except N.NativeError as e:
            if e.code != N.RS_E_ARG:
                raise
        plan.corrupt(stream)  # the no-lookup form's Verify rows compare junk: clear
        plan.launch(stream)
        if plan.corrupt(stream):
            raise SystemExit(f"{name} plan relaunched after its ceilings flagged corruption")
        out[name] = ms
    return out


def layout_ab(k, m, S, B, dev, present, stream, tune, pitch=None):
    """The same encode and decode in two more layouts, timed in this process after the
    bench's own plans: 'pitch' (256-B shard pitch, each stripe's n shards in one block, the
    bench layout of rounds 1-3; decode in place) and 'readall' (upstream Split of an
    io.ReadAll body per object: data at pitch S in the body, parity in AllocAligned buffers;
    decode into fresh buffers, as Reconstruct allocates the missing shards). Each a second
    batch, its plans tuned as the bench's are, mean kernel time of 20 event-timed launches
    after >= 30 ms of warmup each (_launch_ms)."""
    from callfs_amd.device import Plan, StripeBatch, _aligned_empty
    out = {}
    erase = [i for i in range(k + m) if not present[i]]
    for layout in ("pitch", "readall"):
        sb = StripeBatch(k, m, S, B, dev, layout=layout,
                         pitch=pitch if layout == "pitch" else None)
        sb.fill_random(0x5EED)
        enc = Plan.for_batch(sb)
        rebuilt = None
        if layout == "readall":
            rebuilt = _aligned_empty((B, len(erase), sb.par_pitch), 256, dev)
            ptrs = sb.pointers()
            for b in range(B):
                for j, i in enumerate(erase):
                    ptrs[b * (k + m) + i] = rebuilt[b, j].data_ptr()
            dec = Plan(k, m, S, B, ptrs, present=present)
        else:
            dec = Plan.for_batch(sb, present=present)
        enc.launch(stream)
        orders = ({"encode": enc.tune(stream=stream), "decode": dec.tune(stream=stream)}
                  if tune else None)
        r = out[layout] = {"tile_order": orders}
        for name, plan in (("encode", enc), ("decode", dec)):
            ms = _launch_ms(lambda evs: plan.launch(stream, events=evs), stream)
            r[name + "_frac"] = round(plan.bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        if dec.corrupt(stream):
            raise SystemExit(f"{layout}-layout decode flagged corruption")
        if rebuilt is not None and not torch.equal(rebuilt[:, :, :S], sb.gather()[:, erase]):
            raise SystemExit("readall-layout decode rebuilt wrong bytes")
        enc.close()
        dec.close()
        del sb, rebuilt
        torch.cuda.empty_cache()
    out["note"] = ("kernel-time fractions of 8 TB/s, same workload, same process: the bench "
                   "layout ('planar') against each stripe's data and parity in one block "
                   "('pitch') and upstream Split of an io.ReadAll body ('readall'); DESIGN.md §4")
    return out


def load_traffic(path, cfg):
    """PMC-measured HBM bytes per encode / decode launch for this exact config."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None, None
    if t.get("config") != cfg:
        return None, None, None
    return (t.get("encode_bytes_per_launch"), t.get("decode_bytes_per_launch"),
            os.path.relpath(path, HERE))


def ceiling_entry(ceil, name, nbytes, achieved):
    """roofline.copy_ceiling: the plan's bytes over (read-streams-alone time +
    write-streams-alone time), both measured live on the same grid and order."""
    if not ceil:
        return None
    ms = ceil[name]
    gbs = nbytes / ((ms["read"] + ms["write"]) * 1e-3) / 1e9
    return {"kernel": ("rs_stream_read + rs_stream_write: the launch's read streams alone, "
                       "then its write streams alone (same grid, tile order, nt 16-B "
                       "accesses); bytes / summed time"),
            "achieved": round(gbs, 1), "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4),
            "frac": round(achieved / gbs, 4),
            "read_ms": round(ms["read"], 4), "write_ms": round(ms["write"], 4)}


def nolookup_entry(ceil, name, nbytes, achieved):
    """The production kernel's no-lookup form (same loads, stores, grid, order); timed with
    the A/B build of the library only."""
    if not ceil or "nolookup" not in ceil[name]:
        return None
    gbs = nbytes / (ceil[name]["nolookup"] * 1e-3) / 1e9
    return {"kernel": "rs_apply_lds NOMATH form (lookups replaced by one XOR per dword)",
            "achieved": round(gbs, 1), "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4),
            "frac": round(achieved / gbs, 4), "ms": round(ceil[name]["nolookup"], 4)}


def main(argv=None):
    args = parse_args(argv)
    rank, world, local = dist_env()
    if args.gpus != world:
        # one process per GPU: N > 1 comes from torch.distributed.run (WORLD_SIZE)
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}: launch N > 1 as "
                         f"python -m torch.distributed.run --nproc-per-node {args.gpus} "
                         f"bench.py --gpus {args.gpus}")
    # one GPU per rank on a full node; ranks beyond the device count share devices
    # (device_count() does not initialise HIP), which lets a 1-GPU box rehearse N > 1
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from callfs_amd.device import Plan, StripeBatch

    k, m, S, B = args.k, args.m, args.shard_bytes, args.stripes
    if B is None:
        B = 256
        if args.object_bytes:  # configs[3]: 1 GiB objects -> 11 of them at N = 1
            B = max(1, min(256, (16 << 30) // (-(-args.object_bytes // k) * (k + m))))
    scaling, S_obj = "weak", None
    if args.object_bytes:
        # configs[3]: each rank owns a 256-B-aligned byte-column slice of every object
        from callfs_amd.sharding import column_slices
        S_obj = -(-args.object_bytes // k)
        S = column_slices(S_obj, world)[rank][1]
        scaling = "strong"
    erase = sorted({int(x) for x in args.erase.split(",") if x != ""})
    present = [i not in erase for i in range(k + m)]

    layout = args.split_layout or args.layout
    sb = StripeBatch(k, m, S, B, dev, layout=layout,
                     pitch=args.pitch if layout in ("planar", "pitch") else None)
    sb.fill_random(0xCA11F5 + rank)
    enc = Plan.for_batch(sb)
    # decode into fresh buffers (layout planar or readall, --decode-into fresh): the erased
    # shards are rebuilt into their own region, as reedsolomon's Reconstruct allocates the
    # missing shards of a download (codec.go:55) instead of writing over survivors'
    # neighbours; otherwise into the erased shards' own slots of the batch
    fresh = layout in ("planar", "readall") and args.decode_into == "fresh" and erase
    rebuilt = None
    if fresh:
        from callfs_amd.device import _aligned_empty
        rebuilt = _aligned_empty((B, len(erase), sb.par_pitch), 256, dev)
        ptrs = sb.pointers()
        for b in range(B):
            for j, i in enumerate(erase):
                ptrs[b * (k + m) + i] = rebuilt[b, j].data_ptr()
        dec = Plan(k, m, S, B, ptrs, present=present, device=local)
    else:
        dec = Plan.for_batch(sb, present=present)
    stream = torch.cuda.current_stream(dev)

    def rebuilt_ok():
        want = sb.gather()[:, erase]
        return torch.equal(rebuilt[:, :, :S], want)

    # untimed device-side round-trip check: encode, erase, decode, compare
    enc.launch(stream)
    if fresh:
        rebuilt.zero_()
        dec.launch(stream)
        if dec.corrupt(stream) or not rebuilt_ok():
            raise SystemExit("device round trip failed")
    else:
        ref = sb.gather()
        for i in erase:
            sb.zero_shard(i)
        dec.launch(stream)
        if dec.corrupt(stream) or not torch.equal(sb.gather(), ref):
            raise SystemExit("device round trip failed")
        del ref

    # untimed: pick each plan's tile order on this box (the outputs are recomputed to the
    # same bytes; DESIGN.md §6.2 "Tile order"). Tuning is optional: if it fails the plans
    # keep the rule's forms and the line says why (config.tune_error)
    tune_error = None
    try:
        orders = ({"encode": enc.tune(stream=stream), "decode": dec.tune(stream=stream)}
                  if args.tune else None)
    except N.NativeError as e:
        orders, tune_error = None, str(e)[:200]
        enc.set_orders(["none"] * len(enc.forms()))
        dec.set_orders(["none"] * len(dec.forms()))

    for _ in range(args.warmup):
        enc.launch(stream)
        dec.launch(stream)

    # per step: encode start / stop, decode start / stop, recorded by the kernel dispatches
    # (rs_plan_launch_timed); each recorded once here so the HIP events exist
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    for row in ev:
        for e in row:
            e.record(stream)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        enc.launch(stream, events=(ev[s][0], ev[s][1]))
        dec.launch(stream, events=(ev[s][2], ev[s][3]))
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    barrier()
    torch.cuda.synchronize(dev)

    el = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el[0])

    enc_all = sorted(e[0].elapsed_time(e[1]) for e in ev)
    dec_all = sorted(e[2].elapsed_time(e[3]) for e in ev)
    enc_ms = sum(enc_all) / args.steps
    dec_ms = sum(dec_all) / args.steps
    user_step = 2 * B * k * (S_obj if S_obj else S * world)
    value = args.steps * user_step / elapsed / 2**30

    if dec.corrupt(stream):
        raise SystemExit("verify flagged corruption during the timed run")
    if fresh:
        rebuilt.zero_()
        dec.launch(stream)
        if not rebuilt_ok():
            raise SystemExit("rebuilt shards differ from the originals after the timed run")
    ceil = plan_ceilings(enc, dec, stream) if args.ceiling else None
    cfg = {"k": k, "m": m, "shard_bytes": S, "stripes": B}
    if layout != "pitch":
        cfg["layout"] = layout
    traffic, dec_traffic, tsrc = load_traffic(args.traffic, {**cfg, "erase": erase})
    achieved = enc.bytes / (enc_ms * 1e-3) / 1e9
    dec_achieved = dec.bytes / (dec_ms * 1e-3) / 1e9
    verify_rows = max(0, (k + m - len(erase)) - k)  # present parity beyond the first k
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: seeded uniform random bytes generated on device",
        "config": {
            "workload": (f"RS({k},{m}) device-resident encode + decode(erase {erase}), "
                         + (f"{B} objects of {args.object_bytes} B split by byte columns over "
                            f"{world} GPU(s)" if S_obj else f"{S} B shards, {B} stripes per GPU")
                         + ({"split": ", upstream Split layout (pitch = S, contiguous objects)",
                             "readall": ", upstream Split layout of an io.ReadAll body (data "
                                        "shards at pitch = S in the body, parity in 64-B "
                                        "AllocAligned buffers)",
                             "planar": ", 256-B shard pitch, data and parity shards in two "
                                       "regions"}.get(layout, ""))),
            **cfg,
            "erase": erase,
            "decode_into": "fresh buffers (a region of their own)" if fresh else "the batch",
            # decode re-verifies only the present parity beyond the first k (a9): none
            # when exactly k shards survive, as with the default 4-of-14 erasure
            "decode_verify_rows": verify_rows,
            # per launch group, chosen by rs_plan_tune before the warmup (None: the rule)
            "tile_order": orders,
            **({"tune_error": tune_error} if tune_error else {}),
            # the kernel form each launch group ran in the timed steps (rs_plan_forms: a tile
            # order of the nibble-table kernels, or "bs-*" for the bit-sliced ones)
            "forms": {"encode": enc.forms(), "decode": dec.forms()},
            "parallelism": (f"byte-column slices over {world} GPU(s), no collective" if S_obj
                            else f"stripes sharded over {world} GPU(s), no collective"),
        },
        "encode_gib_s": round(world * B * k * S / (enc_ms * 1e-3) / 2**30, 2),
        "decode_gib_s": round(world * B * k * S / (dec_ms * 1e-3) / 2**30, 2),
        "encode_ms": round(enc_ms, 4),
        "decode_ms": round(dec_ms, 4),
        # wall time per step not inside either plan's kernels: the stream's gaps between
        # dependent launches (and the host loop, when it falls behind)
        "launch_gap_ms": round(elapsed * 1e3 / args.steps - enc_ms - dec_ms, 4),
        # median and min per launch beside the mean the roofline uses
        "encode_ms_median_min": [round(enc_all[len(enc_all) // 2], 4), round(enc_all[0], 4)],
        "decode_ms_median_min": [round(dec_all[len(dec_all) // 2], 4), round(dec_all[0], 4)],
        "roofline": {
            "bound": "hbm",
            "kernel": kernel_label(enc, k) + " (encode plan)",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": tsrc,
            "algorithmic_bytes_per_launch": enc.bytes,
            # also against measured ceilings of the same traffic, live
            "copy_ceiling": ceiling_entry(ceil, "encode", enc.bytes, achieved),
            "nolookup": nolookup_entry(ceil, "encode", enc.bytes, achieved),
        },
        "roofline_decode": {
            "bound": "hbm",
            "kernel": kernel_label(dec, k) + " (decode plan)",
            "achieved": round(dec_achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(dec_achieved / HBM_PEAK_GBS, 4),
            "traffic": dec_traffic,
            "algorithmic_bytes_per_launch": dec.bytes,
            "copy_ceiling": ceiling_entry(ceil, "decode", dec.bytes, dec_achieved),
            "nolookup": nolookup_entry(ceil, "decode", dec.bytes, dec_achieved),
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        visible = len(os.sched_getaffinity(0))
        threads = args.cpu_threads or max(1, min(CPU_SHARE, visible))
        line["cpu_baseline"] = cpu_baseline(sb, k, m, erase, args.cpu_seconds,
                                            args.cpu_working_set, threads, all_threads=visible,
                                            rebuilt=rebuilt)
        line["cpu_baseline"]["cores_visible"] = visible
        if threads < visible:
            line["cpu_baseline"]["threads_note"] = (
                f"{threads} of {visible} visible cores: the GPU box's CPU share per GPU is "
                f"{CPU_SHARE} (its affinity mask shows the whole host); --cpu-threads "
                "overrides")
    wrong = None
    if layout == "planar" and args.layout_ab and world == 1 and not S_obj:
        # (one process only: a second resident batch beside the first; freed buffers first)
        del rebuilt
        torch.cuda.empty_cache()
        try:
            line["layout_ab"] = layout_ab(k, m, S, B, dev, present, stream, args.tune, args.pitch)
            line["layout_ab"]["planar"] = {"encode_frac": line["roofline"]["frac"],
                                           "decode_frac": line["roofline_decode"]["frac"]}
        except RuntimeError as e:  # e.g. an allocation failure: recorded, not at the cost of the line
            line["layout_ab"] = {"error": str(e)[:300]}
        except SystemExit as e:  # a flagged decode or wrong bytes: printed with the line, then fatal
            line["layout_ab"] = {"error": str(e)[:300]}
            wrong = e
    if rank == 0:
        print(json.dumps(line), flush=True)
    enc.close()
    dec.close()
    if world > 1:
        torch.distributed.destroy_process_group()
    if wrong is not None:
        raise wrong


if __name__ == "__main__":
    main()
