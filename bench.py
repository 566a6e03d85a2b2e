#!/usr/bin/env python3
"""Benchmark of the MI355X RLE block codec (BASELINE.json metric: GiB/s RLE encode+decode,
device-resident, batched).

One step = one pass of the hot path over one batch resident in HBM: a batched encode launch
(RLEcompress, src/rleCompression.c:9-45) followed by a batched decode launch of its output
(RLEdecompress, src/rleCompression.c:47-62).  With N > 1 ranks (one process per GPU,
torch.distributed over RCCL) the global batch is sharded round-robin (buffer i -> rank i % N)
and each step also all-gathers the per-buffer compressed sizes over xGMI and scans them into
global stream offsets; payloads never leave their GPU.

value = uncompressed bytes round-tripped by all ranks / max-over-ranks wall time of K steps.
Default workload: BASELINE configs[1], 4096 x 4 KiB synthetic buffers per GPU (random / zero).

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg1|dec64k|mixed|cfg3]
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "c-filestorage-server-and-client_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rle_mi355x as R  # noqa: E402
import shard  # noqa: E402

METRIC = "GiB/s RLE encode+decode, device-resident, batched 4–256 KiB buffers"
GIB = float(1 << 30)
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def xs64(s):
    s ^= (s << 13) & 0xFFFFFFFFFFFFFFFF
    s ^= s >> 7
    s ^= (s << 17) & 0xFFFFFFFFFFFFFFFF
    return s


def set_host_wait(mode, device):
    """How the host thread waits in hipDeviceSynchronize / hipStreamSynchronize: "spin"
    (hipDeviceScheduleSpin) or "yield" (hipDeviceScheduleYield), set before the device is first
    used; "auto" leaves the runtime's default.  Returns the mode applied (or an error note)."""
    flags = {"spin": 1, "yield": 2}.get(mode)
    if flags is None:
        return "auto"
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch already loaded (same soname)
    rc = hip.hipSetDevice(ctypes.c_int(device)) or hip.hipSetDeviceFlags(ctypes.c_uint(flags))
    return mode if rc == 0 else f"{mode} (hipSetDeviceFlags rc={rc})"


def mixed_size(i):
    """configs[2] size rule (same as oracle/ref_bench.c --size 0): log-uniform 4 KiB..1 MiB, half
    of them with a non-power-of-two remainder."""
    s = (0x9E3779B97F4A7C15 + i + 0x5151) & 0xFFFFFFFFFFFFFFFF
    s = xs64(s)
    r = s
    U = 1 << (12 + r % 9)
    if (r >> 8) & 1:
        s = xs64(s)
        U += (s >> 16) % U
    return U


WORKLOADS = {
    # name: (buffers per GPU, size(global index) or fixed, kind(local index), description)
    "cfg1": dict(n=4096, size=4096, kinds=(1, 0), ref_kinds="1,0",
                 desc="configs[1]: 4096 x 4 KiB synthetic buffers per GPU (random / zero alternating), "
                      "encode+decode round trip"),
    "dec64k": dict(n=16384, size=65536, kinds=(0, 1, 2, 3), ref_kinds="0,1,2,3",
                   desc="16384 x 64 KiB per GPU (zero / random / runs50 / runs90), encode+decode round trip"),
    # per-kind 64 KiB batches (profiling: tile cost per data kind)
    "k64_zero": dict(n=16384, size=65536, kinds=(0,), ref_kinds="0", desc="16384 x 64 KiB zero"),
    "k64_random": dict(n=16384, size=65536, kinds=(1,), ref_kinds="1", desc="16384 x 64 KiB random"),
    "k64_runs50": dict(n=16384, size=65536, kinds=(2,), ref_kinds="2", desc="16384 x 64 KiB runs50"),
    "k64_runs90": dict(n=16384, size=65536, kinds=(3,), ref_kinds="3", desc="16384 x 64 KiB runs90"),
    # configs[1] shape with one data kind (profiling: per-SIMD balance of the mixed batch)
    "c4k_random": dict(n=4096, size=4096, kinds=(1,), ref_kinds="1", desc="4096 x 4 KiB random"),
    "c4k_zero": dict(n=4096, size=4096, kinds=(0,), ref_kinds="0", desc="4096 x 4 KiB zero"),
    "c4k_runs50": dict(n=4096, size=4096, kinds=(2,), ref_kinds="2", desc="4096 x 4 KiB runs50"),
    "s4k_mix": dict(n=65536, size=4096, kinds=(0, 1, 2, 3), ref_kinds="0,1,2,3", desc="65536 x 4 KiB zero/random/runs50/runs90"),
    "one4m": dict(n=1, size=4 << 20, kinds=(1,), ref_kinds="1", desc="1 x 4 MiB random (one large file)"),
    "one64m": dict(n=1, size=64 << 20, kinds=(2,), ref_kinds="2", desc="1 x 64 MiB runs50 (one large file)"),
    "mixed": dict(n=1024, size=None, kinds=(0, 1, 2, 3), ref_kinds="0,1,2,3",
                  desc="configs[2]: 1024 mixed 4 KiB-1 MiB buffers per GPU (zero / random / runs50 / runs90)"),
    "cfg3": dict(n=131072, size=65536, kinds=(0, 1, 2, 3), ref_kinds="0,1,2,3",
                 desc="configs[3] shard: 131072 x 64 KiB per GPU (1 M x 64 KiB over 8 GPUs), round-robin"),
}


class Batch:
    """One rank's shard of a synthetic batch, resident in HBM, with compressed and decoded slots."""

    def __init__(self, wl, rank, world, dev):
        n = wl["n"]
        kinds = wl["kinds"]
        gidx = [k * world + rank for k in range(n)]   # shard.shard_indices(n * world, rank, world)
        sizes = [wl["size"] if wl["size"] else mixed_size(i) for i in gidx]
        pad = int(os.environ.get("RLE_BENCH_PAD", "0"))   # layout experiments: spare bytes per buffer
        offs, total = R.layout(sizes, pad=pad)
        coffs, ctotal = R.compressed_slots(sizes, pad=pad)
        self.c_cap = ctotal
        self.ws_enc = R.seg_workspace(n, sum(sizes), dev)
        self.ws_dec = R.seg_workspace(n, ctotal, dev)
        i64 = lambda v: torch.tensor(v, dtype=torch.int64, device=dev)
        self.n = n
        self.sizes = sizes
        # the batch's largest buffer (the sized entry points pick the cooperative small-buffer
        # kernels from it); the largest compressed size is known once the batch has been encoded
        self.max_u = max(sizes)
        self.max_c = R.max_compressed_size(self.max_u)
        self.u_bytes = sum(sizes)
        self.offs, self.lens = i64(offs), i64(sizes)
        self.coffs = i64(coffs)
        self.clen = torch.zeros(n, dtype=torch.int64, device=dev)
        self.status = torch.zeros(n, dtype=torch.int32, device=dev)
        # zero-filled, so the padding between buffers (sizes not a multiple of 16, RLE_BENCH_PAD) is
        # equal in d_in and d_out and the whole-arena comparison checks only the decoded bytes
        self.d_in = torch.zeros(total, dtype=torch.uint8, device=dev)
        self.d_c = torch.empty(ctotal, dtype=torch.uint8, device=dev)
        self.d_out = torch.zeros(total, dtype=torch.uint8, device=dev)
        kind_t = torch.tensor([kinds[k % len(kinds)] for k in range(n)], dtype=torch.int32, device=dev)
        R.gen_synthetic(self.d_in, self.offs, self.lens, kind_t, i64(gidx))
        torch.cuda.synchronize()

    seg = False   # True: the segmented (several waves per buffer) entry points

    def encode(self, stream=None):
        if self.seg:
            R.encode_batch_seg(self.d_in, self.offs, self.lens, self.d_c, self.coffs, self.clen, self.status,
                               total_in_bytes=self.u_bytes, workspace=self.ws_enc, stream=stream)
        else:
            R.encode_batch(self.d_in, self.offs, self.lens, self.d_c, self.coffs, self.clen, self.status,
                           stream=stream, max_len=self.max_u)

    def decode(self, stream=None):
        if self.seg:
            R.decode_batch_seg(self.d_c, self.coffs, self.clen, self.d_out, self.offs, self.lens, None, self.status,
                               total_in_bytes=self.c_cap, workspace=self.ws_dec, stream=stream)
        else:
            R.decode_batch(self.d_c, self.coffs, self.clen, self.d_out, self.offs, self.lens, None, self.status,
                           stream=stream, max_in_len=self.max_c, max_out_len=self.max_u)

    def calibrate(self):
        """After an encode: the largest compressed size, as a file server knows from its stored sizes."""
        torch.cuda.synchronize()
        self.max_c = int(self.clen.max().item())


def time_kernels(fn, reps, stream):
    """Average duration of fn's launch: reps launches back to back on the stream the kernel runs on,
    between one pair of HIP events (an event pair around every launch would add its own dispatch,
    ~2 us, to each; back to back, each launch carries only its share of the kernel boundaries)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def copy_ceiling(B, alg, reps, stream):
    """Practical ceiling: a device-to-device copy that moves the same algorithmic
    bytes as one codec launch (alg / 2 read + alg / 2 written, HBM to HBM), timed like the kernels.
    Runs after the round trip was verified; it overwrites the front of d_out with d_in's bytes, which
    is the decoded content anyway."""
    n = min(alg // 2, B.d_in.numel(), B.d_out.numel())
    src, dst = B.d_in[:n], B.d_out[:n]
    t = time_kernels(lambda: dst.copy_(src), reps, stream)
    return {"GBps": round(2 * n / t / 1e9, 2), "frac": round(2 * n / t / 1e9 / HBM_PEAK_GBPS, 4), "bytes": 2 * n,
            "us": round(t * 1e6, 3), "op": "torch copy_ (hipMemcpyAsync device to device)"}


def cpu_baseline(wl, seconds, threads, flavor):
    """The reference codec (src/rleCompression.c compiled unchanged by oracle/Makefile) timed on this
    host's cores on the same synthetic batch, repeated passes for a bounded sample."""
    exe = os.path.join(REPO, "oracle", "_ref", f"ref_bench_{flavor}")
    if not os.path.exists(exe):
        return None
    size = wl["size"] if wl["size"] else 0
    cmd = [exe, "--kinds", wl["ref_kinds"], "--size", str(size), "--count", str(wl["n"]), "--threads",
           str(threads), "--seconds", str(seconds)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds * 4 + 120)
    if r.returncode != 0:
        print(f"cpu baseline failed: {r.stderr}", file=sys.stderr)
        return None
    return json.loads(r.stdout.strip().splitlines()[-1])


def load_pmc(workload):
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p)).get(workload)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfg1", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-north-star", action="store_true")
    ap.add_argument("--no-concurrent", action="store_true",
                    help="skip the informational two-stream figure (profiling runs: its overlapped launches "
                         "would enter the per-kernel averages)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    sched = set_host_wait(os.environ.get("RLE_BENCH_SCHED", "auto"), local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    wl = WORKLOADS[args.workload]
    stream = torch.cuda.current_stream()

    B = Batch(wl, rank, world, dev)
    # N > 1: the one exchange step -- each step's compressed sizes all-gathered over RCCL and
    # scanned into global stream offsets -- runs on its own stream, off the codec's critical path.
    # The sizes are copied into one of two buffers, so a gather may overlap the decode of its own
    # step and the whole next step; a step waits only for the gather of two steps back (buffer
    # reuse).  Every gather still completes inside the timed region (the final synchronize).
    comm = torch.cuda.Stream(device=dev) if world > 1 else None
    sizes = [torch.empty_like(B.clen) for _ in range(2)] if world > 1 else None
    gathered = [torch.cuda.Event() for _ in range(2)] if world > 1 else None
    nstep = [0]

    # N > 1: the exchange as one library call per step on the codec's stream (csrc/rle_dist.hip)
    # when every rank's RCCL communicator comes up; else the torch calls below, on a side stream
    # (host-bound: tools/exchange_cost.py)
    xch = shard.NativeExchange(B.n, world, rank, dev) if world > 1 else None
    if xch is not None and not xch.ok and rank == 0:
        print(f"native exchange unavailable ({xch.error}); torch calls", file=sys.stderr)

    def step():
        B.encode(stream)
        if xch is not None and xch.ok:
            xch.step(B.clen, stream)
        elif world > 1:
            k = nstep[0] % 2
            nstep[0] += 1
            stream.wait_event(gathered[k])
            sizes[k].copy_(B.clen)
            comm.wait_stream(stream)
            with torch.cuda.stream(comm):
                shard.global_offsets(sizes[k], world)
                gathered[k].record(comm)
        B.decode(stream)

    B.encode(stream)
    B.calibrate()
    # verified on one step first, so that the W warmup steps run right before the timed region (host
    # work between them, with the GPU idle, made the first timed step ~50 us slower: tools/step_profile.py)
    step()
    torch.cuda.synchronize()
    ok = bool(torch.equal(B.d_out, B.d_in)) and int(B.status.abs().sum().item()) == 0
    c_bytes = int(B.clen.sum().item())
    u_local = B.u_bytes
    for _ in range(max(1, args.warmup)):
        step()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
        ut = torch.tensor([u_local], dtype=torch.int64, device=dev)
        dist.all_reduce(ut, op=dist.ReduceOp.SUM)
        total_u = int(ut.item())
    else:
        total_u = u_local

    # per-kernel durations (HIP events on the launch stream), algorithmic bytes = U + C per launch
    reps = max(10, min(args.steps, 50))
    t_enc = time_kernels(lambda: B.encode(stream), reps, stream)
    t_dec = time_kernels(lambda: B.decode(stream), reps, stream)
    alg = u_local + c_bytes
    # GBps: algorithmic bytes (U + C) per second, the roofline numerator; U_GiBps: uncompressed bytes
    # per second (SURVEY.md 8(d) reports both), also for the round trip
    kern = {"encode": {"us": t_enc * 1e6, "GBps": alg / t_enc / 1e9, "U_GiBps": u_local / t_enc / GIB},
            "decode": {"us": t_dec * 1e6, "GBps": alg / t_dec / 1e9, "U_GiBps": u_local / t_dec / GIB},
            "roundtrip": {"us": (t_enc + t_dec) * 1e6, "U_GiBps": u_local / (t_enc + t_dec) / GIB}}
    dom = "encode" if t_enc >= t_dec else "decode"
    pmc = load_pmc(args.workload)
    traffic = pmc.get(dom) if isinstance(pmc, dict) else None
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(kern[dom]["GBps"], 2), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(kern[dom]["GBps"] / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "alg_bytes_per_launch": alg, "copy_ceiling": copy_ceiling(B, alg, reps, stream)}

    # Informational, not `value`: the same round trips with two batches in flight on two streams, as
    # the drop-in runs when the server's worker threads (one HIP stream each) call it concurrently.
    conc = None
    if rank == 0 and world == 1 and B.u_bytes <= (256 << 20) and args.steps > 0 and not args.no_concurrent:
        B2 = Batch(wl, rank, world, dev)
        B2.encode(stream)
        B2.calibrate()
        ss = [stream, torch.cuda.Stream(device=dev)]
        pair = [B, B2]
        for k in range(4):
            pair[k % 2].encode(ss[k % 2])
            pair[k % 2].decode(ss[k % 2])
        torch.cuda.synchronize()
        t0c = time.perf_counter()
        for k in range(2 * args.steps):
            pair[k % 2].encode(ss[k % 2])
            pair[k % 2].decode(ss[k % 2])
        torch.cuda.synchronize()
        dtc = time.perf_counter() - t0c
        conc = {"streams": 2, "value": round(B.u_bytes * 2 * args.steps / dtc / GIB, 3), "unit": "GiB/s",
                "us_per_roundtrip": round(dtc / (2 * args.steps) * 1e6, 3),
                "verified": bool(torch.equal(B2.d_out, B2.d_in)),
                "note": "two independent batches, each round trip on its own stream (the drop-in's per-thread "
                        "streams); `value` is one batch after another on one stream"}
        del B2
        torch.cuda.empty_cache()

    north = None
    if rank == 0 and world == 1 and not args.no_north_star and args.workload != "dec64k":
        del B
        torch.cuda.empty_cache()
        N = Batch(WORKLOADS["dec64k"], 0, 1, dev)
        N.encode(stream)
        N.calibrate()
        nc = int(N.clen.sum().item())
        td = time_kernels(lambda: N.decode(stream), 20, stream)
        te = time_kernels(lambda: N.encode(stream), 20, stream)
        nok = bool(torch.equal(N.d_out, N.d_in))
        nalg = N.u_bytes + nc
        ncopy = copy_ceiling(N, nalg, 20, stream)
        north = {"workload": WORKLOADS["dec64k"]["desc"], "decode_us": td * 1e6,
                 "decode_U_GiBps": N.u_bytes / td / GIB, "encode_U_GiBps": N.u_bytes / te / GIB,
                 "decode_GBps": nalg / td / 1e9, "decode_frac": round(nalg / td / 1e9 / HBM_PEAK_GBPS, 4),
                 "encode_GBps": nalg / te / 1e9, "u_bytes": N.u_bytes, "c_bytes": nc, "verified": nok,
                 "copy_ceiling": ncopy}
        del N
        torch.cuda.empty_cache()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = min(16, os.cpu_count() or 1)
        r0 = cpu_baseline(wl, args.cpu_seconds, threads, "O0")
        r2 = cpu_baseline(wl, max(2.0, args.cpu_seconds / 2), threads, "O2")
        if r0:
            cpu = {"value": round(r0["rt_gibs"], 4), "unit": "GiB/s", "cores": threads, "kind": "reference",
                   "sample": f"reference src/rleCompression.c compiled unchanged with its Makefile flags "
                             f"(-Wall -g -std=c99), {threads} pthreads, repeated passes over the same batch for "
                             f"{args.cpu_seconds:.0f} s ({r0['buffers']} buffers, {r0['u_bytes']} bytes)",
                   "c_batch_match": r0["c_batch"] == c_bytes,
                   "O2": round(r2["rt_gibs"], 4) if r2 else None}

    if rank == 0:
        value = total_u * args.steps / elapsed / GIB
        out = {"metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
               "config": {"workload": wl["desc"], "buffers_per_gpu": wl["n"],
                          "buffer_bytes": wl["size"] or "mixed 4 KiB-2 MiB",
                          "u_bytes_per_gpu": total_u // world, "c_bytes_rank0": c_bytes,
                          "parallelism": f"shard round-robin over {world} GPU(s)" +
                                         (", RCCL all-gather of sizes" if world > 1 else "") +
                                         ((" (one library call per step)" if xch.ok else " (torch calls)")
                                          if xch is not None else "")},
               "verified_bit_exact_roundtrip": ok, "host_wait": sched, "kernels": kern, "roofline": roofline, "cpu_baseline": cpu,
               "north_star_dec64k": north, "concurrent_streams": conc}
        print(json.dumps(out))
    if xch is not None:
        torch.cuda.synchronize()
        xch.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
