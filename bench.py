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

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg1|dec64k|mixed|cfg3|...]

`--gpus N` with N > 1 and no WORLD_SIZE in the environment starts the N rank processes itself
(127.0.0.1 rendezvous) before anything touches the GPU; under torch.distributed.run each rank
reads RANK / LOCAL_RANK / WORLD_SIZE.  `--dry-run` runs the same rank loop on the CPU over gloo with
the codec launches left out (sizes come from a closed form): it exercises the rank spawn, the
process group, the exchange fallback, the barriers and the max-over-ranks timing, never the GPU.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "c-filestorage-server-and-client_amd")]

# The drop-in's background start-up (csrc/rle_dropin.cpp preinit_main) builds warm per-thread
# contexts for server processes; bench uses only the batched device API, so it stays off here and
# runs no GPU work beside the timed loop.
os.environ.setdefault("RLE_MI355X_PREINIT", "0")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rle_mi355x as R  # noqa: E402  (loads nothing until first use)
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
    # two kinds side by side (profiling: does a store-bound kind overlap a run-heavy one)
    "k64_z50": dict(n=16384, size=65536, kinds=(0, 2), ref_kinds="0,2", desc="16384 x 64 KiB zero / runs50"),
    # configs[1] shape with one data kind (profiling: per-SIMD balance of the mixed batch)
    "c4k_random": dict(n=4096, size=4096, kinds=(1,), ref_kinds="1", desc="4096 x 4 KiB random"),
    "c4k_zero": dict(n=4096, size=4096, kinds=(0,), ref_kinds="0", desc="4096 x 4 KiB zero"),
    "c4k_runs50": dict(n=4096, size=4096, kinds=(2,), ref_kinds="2", desc="4096 x 4 KiB runs50"),
    # a quarter of a wave per SIMD (profiling with RLE_MI355X_COOP=0: one lone wave's walk)
    "c4k_random_q": dict(n=256, size=4096, kinds=(1,), ref_kinds="1", desc="256 x 4 KiB random"),
    "c4k_zero_q": dict(n=256, size=4096, kinds=(0,), ref_kinds="0", desc="256 x 4 KiB zero"),
    "s4k_mix": dict(n=65536, size=4096, kinds=(0, 1, 2, 3), ref_kinds="0,1,2,3", desc="65536 x 4 KiB zero/random/runs50/runs90"),
    "one4m": dict(n=1, size=4 << 20, kinds=(1,), ref_kinds="1", desc="1 x 4 MiB random (one large file)"),
    "one64m": dict(n=1, size=64 << 20, kinds=(2,), ref_kinds="2", desc="1 x 64 MiB runs50 (one large file)"),
    # configs[2]'s 1 MiB end (the sweep's last rows; segmented-path A/B)
    "m1_zero": dict(n=1024, size=1 << 20, kinds=(0,), ref_kinds="0", desc="1024 x 1 MiB zero"),
    "m1_random": dict(n=1024, size=1 << 20, kinds=(1,), ref_kinds="1", desc="1024 x 1 MiB random"),
    "m1_runs50": dict(n=1024, size=1 << 20, kinds=(2,), ref_kinds="2", desc="1024 x 1 MiB runs50"),
    "mixed": dict(n=1024, size=None, kinds=(0, 1, 2, 3), ref_kinds="0,1,2,3",
                  desc="configs[2]: 1024 mixed 4 KiB-1 MiB buffers per GPU (zero / random / runs50 / runs90)"),
    "cfg3": dict(n=131072, size=65536, kinds=(0, 1, 2, 3), ref_kinds="0,1,2,3",
                 desc="configs[3] shard: 131072 x 64 KiB per GPU (1 M x 64 KiB over 8 GPUs), round-robin"),
}


# ---------------------------------------------------------------------------------------- batches
class Batch:
    """One rank's shard of a synthetic batch, resident in HBM, with compressed and decoded slots.
    Two compressed-size vectors alternate between steps (clens[step % 2]), so a step's size exchange
    may still be reading its vector while the next step's encode writes the other one."""

    seg = False   # True: the segmented (several waves per buffer) entry points

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
        self.clens = [torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(2)]
        self.clen = self.clens[0]
        self.status = torch.zeros(n, dtype=torch.int32, device=dev)
        # zero-filled, so the padding between buffers (sizes not a multiple of 16, RLE_BENCH_PAD) is
        # equal in d_in and d_out and the whole-arena comparison checks only the decoded bytes
        self.d_in = torch.zeros(total, dtype=torch.uint8, device=dev)
        self.d_c = torch.empty(ctotal, dtype=torch.uint8, device=dev)
        self.d_out = torch.zeros(total, dtype=torch.uint8, device=dev)
        kind_t = torch.tensor([kinds[k % len(kinds)] for k in range(n)], dtype=torch.int32, device=dev)
        R.gen_synthetic(self.d_in, self.offs, self.lens, kind_t, i64(gidx))
        torch.cuda.synchronize()

    def encode(self, stream=None, slot=0):
        clen = self.clens[slot]
        if self.seg:
            R.encode_batch_seg(self.d_in, self.offs, self.lens, self.d_c, self.coffs, clen, self.status,
                               total_in_bytes=self.u_bytes, workspace=self.ws_enc, stream=stream)
        else:
            R.encode_batch(self.d_in, self.offs, self.lens, self.d_c, self.coffs, clen, self.status,
                           stream=stream, max_len=self.max_u)

    def decode(self, stream=None, slot=0):
        clen = self.clens[slot]
        if self.seg:
            R.decode_batch_seg(self.d_c, self.coffs, clen, self.d_out, self.offs, self.lens, None, self.status,
                               total_in_bytes=self.c_cap, workspace=self.ws_dec, stream=stream)
        else:
            R.decode_batch(self.d_c, self.coffs, clen, self.d_out, self.offs, self.lens, None, self.status,
                           stream=stream, max_in_len=self.max_c, max_out_len=self.max_u)

    def calibrate(self):
        """After an encode: the largest compressed size, as a file server knows from its stored sizes."""
        torch.cuda.synchronize()
        self.max_c = int(self.clen.max().item())

    def verify(self):
        """decode(encode(x)) == x over the whole arena and every status clean."""
        torch.cuda.synchronize()
        return bool(torch.equal(self.d_out, self.d_in)) and int(self.status.abs().sum().item()) == 0


class DryBatch:
    """--dry-run stand-in for Batch (CPU, no codec): the same shard layout, with each buffer's
    "compressed size" a closed form of its global index, so that the exchange's offsets can be
    checked exactly on every rank."""

    seg = False

    def __init__(self, wl, rank, world, dev):
        self.n = wl["n"]
        gidx = torch.arange(self.n, dtype=torch.int64) * world + rank
        self.sizes_t = self.dry_sizes(gidx, wl)
        self.clens = [torch.zeros(self.n, dtype=torch.int64) for _ in range(2)]
        self.clen = self.clens[0]
        self.u_bytes = self.n * (wl["size"] or 4096)

    @staticmethod
    def dry_sizes(gidx, wl):
        U = wl["size"] or 4096
        return (gidx * 2654435761) % (U + U // 2) + 1

    def encode(self, stream=None, slot=0):
        self.clens[slot].copy_(self.sizes_t)

    def decode(self, stream=None, slot=0):
        pass

    def calibrate(self):
        pass

    def verify(self):
        return None   # nothing was encoded


# --------------------------------------------------------------------------------- rank spawning
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n, argv):
    """Start n rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE set, rendezvous on
    127.0.0.1) and wait for them.  This process never touches the GPU.  If a rank fails, the others
    are stopped (they would wait in a collective for it).  Returns the exit code."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    while procs:
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0 and rc == 0:
                rc = c
                print(f"bench: a rank exited with {c}; stopping the others", file=sys.stderr)
                for q in procs:
                    q.terminate()
                deadline = time.time() + 20
                for q in procs:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
        time.sleep(0.05)
    return rc


# ------------------------------------------------------------------------------------ measurement
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
    bytes as one codec launch (alg / 2 read + alg / 2 written, HBM to HBM), timed like the kernels,
    by the library's hand-written 16-byte-per-lane streaming copy (rle_copy_device) and by the
    runtime's hipMemcpyAsync.  Runs after the round trip was verified; it overwrites the front of
    d_out with d_in's bytes, which is the decoded content anyway."""
    n = min(alg // 2, B.d_in.numel(), B.d_out.numel()) & ~15
    src, dst = B.d_in[:n], B.d_out[:n]
    t_k = time_kernels(lambda: R.copy_device(dst, src, n, stream), reps, stream)
    t_r = time_kernels(lambda: dst.copy_(src), reps, stream)
    t = min(t_k, t_r)
    return {"GBps": round(2 * n / t / 1e9, 2), "frac": round(2 * n / t / 1e9 / HBM_PEAK_GBPS, 4), "bytes": 2 * n,
            "us": round(t * 1e6, 3), "kernel_us": round(t_k * 1e6, 3), "memcpy_us": round(t_r * 1e6, 3),
            "op": "the faster of rle_copy_device (16 B per lane, hand-written) and hipMemcpyAsync, device to device"}


def step_kernels(B, reps, stream, loop_gpu_s=None, steps=None, loop_src="timed_loop_events"):
    """Per-kernel durations consistent with the timed steps.  The GPU time of the timed loop itself
    (HIP events on the launch stream around the K timed steps, or around the same K steps run again
    right after the timed region, loop_gpu_s; loop_src says which) is split between the two
    kernels in the ratio of their back-to-back single-kernel times, so encode + decode is the timed
    step's GPU time and never exceeds ms_per_step (round 3 split a separate back-to-back pair run
    after the timed loop, which on the driver box came out 9 % above the step).  Without the loop's
    events (tools that call this directly) the separate pair run is split instead."""
    t_enc1 = time_kernels(lambda: B.encode(stream), reps, stream)
    t_dec1 = time_kernels(lambda: B.decode(stream), reps, stream)
    t_pair = time_kernels(lambda: (B.encode(stream), B.decode(stream)), reps, stream)
    f = t_enc1 / (t_enc1 + t_dec1)
    t_step = loop_gpu_s / steps if loop_gpu_s and steps else t_pair
    return t_step * f, t_step * (1 - f), {"split_of": loop_src if loop_gpu_s and steps else "pair_us",
                                          "timed_loop_gpu_us_per_step": t_step * 1e6, "pair_us": t_pair * 1e6,
                                          "encode_alone_us": t_enc1 * 1e6, "decode_alone_us": t_dec1 * 1e6}


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


# ------------------------------------------------------------------------------------ the exchange
# The exchange mode: "auto" times inline and async on the job's own ranks and keeps the faster.
XMODE_REASON = ("auto: inline and async timed on the job's own ranks before the timed region, the faster kept "
                "(auto_us_per_step); one-rank RCCL rehearsal (DESIGN.md s7, r3b): inline 29.4 us per configs[1] "
                "step against 35.0 (async) and 45.0 (graph); async's overlap of the gather is unmeasured at N > 1 "
                "on this pool's one-GPU boxes")
class Exchange:
    """The N > 1 exchange step of one rank: after a step's encode, its compressed
    sizes are all-gathered and scanned into global stream offsets.  Modes (RLE_BENCH_XMODE):
      inline   (default) one library call (rle_dist_gather_offsets: ncclAllGather + the scan
               kernels) on the codec's stream, between encode and decode -- the measured-faster mode
               (XMODE_REASON);
      async    one library call per step (rle_dist_gather_offsets_async): the gather + scan run on
               a side stream after the step's encode, beside its decode and the next step's encode;
               the codec stream waits only for the previous step's exchange;
      graph    the inline calls captured with the whole timed loop in one HIP graph, the gather of
               step i on a graph branch beside decode i and encode i + 1;
      torch    shard.global_offsets (all_gather_into_tensor + cumsum) on a side stream: the fallback
               when RCCL cannot be resolved on every rank, and the --dry-run (gloo, CPU) path.
    Every rank takes the same mode (flags all-reduced with MIN before any rank commits)."""

    def __init__(self, B, world, rank, dev, dry, xmode):
        self.B, self.world, self.rank, self.dev, self.dry = B, world, rank, dev, dry
        self.mode, self.error, self.xch = "torch", None, None
        self.nstep = 0
        if not dry:
            self.comm = torch.cuda.Stream(device=dev)
            self.gathered = [torch.cuda.Event() for _ in range(2)]
            try:
                self.xch = shard.NativeExchange(B.n, world, rank, dev)
                if self.xch.ok:
                    self.mode = xmode
                else:
                    self.error = self.xch.error
            except Exception as e:   # every rank reaches the collective checks inside NativeExchange
                self.error = e
        self.offsets = None

    def run(self, stream, slot):
        """One exchange on the sizes of clens[slot], after the encode issued on `stream`."""
        clen = self.B.clens[slot]
        if self.mode in ("inline", "graph"):
            self.offsets = self.xch.step(clen, stream, slot)
        elif self.mode == "async":
            self.offsets = self.xch.step_async(clen, stream, self.comm, slot)
        elif self.dry:
            self.offsets = shard.global_offsets(clen, self.world)
        else:
            k = slot
            self.comm.wait_stream(stream)
            with torch.cuda.stream(self.comm):
                self.offsets = shard.global_offsets(clen, self.world)
                self.gathered[k].record(self.comm)

    def verify(self, stream):
        """Once, before timing: this rank's exchange result for clens[0] against the torch
        process-group path (shard.global_offsets) -- exact int64 equality."""
        if not self.dry:
            torch.cuda.synchronize()
        ref = shard.global_offsets(self.B.clens[0], self.world)
        if self.dry:
            n, w = self.B.n, self.world
            gidx = torch.arange(n * w, dtype=torch.int64)
            s = DryBatch.dry_sizes(gidx, {"size": self.B.u_bytes // n})
            ok = torch.equal(ref, torch.cumsum(s, 0) - s)
        else:
            torch.cuda.synchronize()
            ok = torch.equal(self.offsets, ref)
        return bool(ok)

    def close(self):
        if self.xch is not None:
            if not self.dry:
                torch.cuda.synchronize()
            self.xch.close()


# ----------------------------------------------------------------------------------- the rank loop
class Loop:
    """The timed loop of one rank: `steps(k)` issues k steps (eager), or replays a captured graph
    of k steps (Exchange mode "graph").  In graph mode step i encodes into clens[i % 2]; the gather of
    step i runs on a branch, beside decode i and encode i + 1, and encode i + 2 (which rewrites
    clens[i % 2]) waits for it.  Without an exchange (one rank) the timed steps are issued eagerly,
    2 launches per step from the host; `plain` (RLE_BENCH_GRAPH=1) captures the k steps (encode i,
    decode i, one after another on one stream) in one HIP graph and the timed region replays it.
    Round 5 measured the replay ~2 % SLOWER than eager issue on every box (driver 787.0
    graph against 804.1 eager), so eager is the headline since round 6 and the replayed form is
    reported beside it (value_graph)."""

    def __init__(self, B, xch, stream, dry):
        self.B, self.xch, self.stream, self.dry = B, xch, stream, dry
        self.graphs = {}
        self.plain = (xch is None and not dry and os.environ.get("RLE_BENCH_GRAPH", "0") == "1")

    def capture_plain(self, k):
        g = torch.cuda.CUDAGraph()
        main = torch.cuda.Stream(device=self.stream.device)
        main.wait_stream(self.stream)
        with torch.cuda.graph(g, stream=main):
            for i in range(k):
                self.B.encode(main, i % 2)
                self.B.decode(main, i % 2)
        self.stream.wait_stream(main)
        torch.cuda.synchronize()
        self.graphs[k] = g

    def one_step(self, slot):
        if self.xch is not None and self.xch.mode == "torch" and not self.dry:
            self.stream.wait_event(self.xch.gathered[slot])   # the side-stream gather still reading clens[slot]
        self.B.encode(self.stream, slot)
        if self.xch is not None:
            self.xch.run(self.stream, slot)
        self.B.decode(self.stream, slot)

    def _issue_pipelined(self, k, main, side):
        done = [None, None]
        for i in range(k):
            slot = i % 2
            if done[slot] is not None:
                main.wait_event(done[slot])
            self.B.encode(main, slot)
            enc = torch.cuda.Event()
            enc.record(main)
            side.wait_event(enc)
            self.xch.run(side, slot)
            done[slot] = torch.cuda.Event()
            done[slot].record(side)
            self.B.decode(main, slot)
        main.wait_stream(side)

    def capture(self, k):
        g = torch.cuda.CUDAGraph()
        main = torch.cuda.Stream(device=self.stream.device)
        side = torch.cuda.Stream(device=self.stream.device)
        main.wait_stream(self.stream)
        with torch.cuda.graph(g, stream=main, capture_error_mode="relaxed"):
            side.wait_stream(main)
            self._issue_pipelined(k, main, side)
        self.stream.wait_stream(main)
        torch.cuda.synchronize()
        self.graphs[k] = g

    def steps(self, k):
        if self.plain:
            if k not in self.graphs:
                self.capture_plain(k)
            self.graphs[k].replay()
            return
        if self.xch is not None and self.xch.mode == "graph":
            if k not in self.graphs:
                self.capture(k)
            self.graphs[k].replay()
            return
        for i in range(k):
            self.one_step(i % 2)


def sync(dry):
    if not dry:
        torch.cuda.synchronize()


def run_rank(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dry = args.dry_run
    wl = WORKLOADS[args.workload]
    # RLE_BENCH_FORCE_EXCHANGE=1 (rehearsal on a one-GPU box): a one-rank process group and the whole
    # N > 1 path -- RCCL communicator, exchange, graph capture, barriers -- at world size 1
    multi = world > 1 or os.environ.get("RLE_BENCH_FORCE_EXCHANGE") == "1"
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
    if dry:
        dev, sched, stream = torch.device("cpu"), "n/a (dry run)", None
        if os.environ.get("RLE_BENCH_DRY_FAIL_RANK") == str(rank):   # tests: a rank that dies before the rendezvous
            sys.exit(3)
        if multi:
            dist.init_process_group("gloo")
        B = DryBatch(wl, rank, world, dev)
    else:
        sched = set_host_wait(os.environ.get("RLE_BENCH_SCHED", "auto"), local)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if multi:
            dist.init_process_group("nccl", device_id=dev)
        stream = torch.cuda.current_stream()
        B = Batch(wl, rank, world, dev)

    xmode = os.environ.get("RLE_BENCH_XMODE", "auto")
    if xmode not in ("auto", "async", "inline", "graph"):
        raise SystemExit(f"RLE_BENCH_XMODE={xmode}: auto, async, inline or graph")
    xch = Exchange(B, world, rank, dev, dry, "inline" if xmode == "auto" else xmode) if multi else None
    if xch is not None and xch.mode == "torch" and not dry and rank == 0:
        print(f"native exchange unavailable ({xch.error}); torch calls", file=sys.stderr)
    loop = Loop(B, xch, stream, dry)

    B.encode(stream)
    B.calibrate()
    # verified on one step first, so that the W warmup steps run right before the timed region (host
    # work between them, with the GPU idle, made the first timed step ~50 us slower: tools/step_profile.py)
    loop.one_step(0)
    sync(dry)
    ok = B.verify()
    offsets_ok = xch.verify(stream) if xch is not None else None
    c_bytes = int(B.clen.sum().item())
    u_local = B.u_bytes
    # the graph (N > 1) is captured here, outside the timed region, and replayed for warmup too
    graph_ok = None
    if xch is not None and xch.mode == "graph":
        try:
            loop.capture(args.steps)
            if args.warmup != args.steps:
                loop.capture(max(1, args.warmup))
            up = 1
        except Exception as e:
            print(f"rank {rank}: graph capture failed ({e}); eager exchange", file=sys.stderr)
            up = 0
        t = torch.tensor([up], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        graph_ok = bool(t.item())
        if not graph_ok:
            xch.mode = "inline"
            loop.graphs.clear()
    if loop.plain:   # (captured here, outside the timed region)
        try:
            loop.capture_plain(args.steps)
            if args.warmup != args.steps:
                loop.capture_plain(max(1, args.warmup))
        except Exception as e:
            print(f"graph capture failed ({e}); eager steps", file=sys.stderr)
            loop.plain = False
            loop.graphs.clear()
    loop.steps(max(1, args.warmup))
    # RLE_BENCH_XMODE=auto (the default): the exchange mode is chosen on this job's own ranks, before
    # the timed region -- K steps inline and K steps async, each timed between barriers, the max over
    # ranks, the faster mode kept (every rank takes the same numbers).  At one rank inline measured
    # faster (XMODE_REASON); at N > 1 the all-gather's latency over xGMI can exceed a step, which
    # async overlaps with the decode and the next encode.  Its result is verified as inline's was.
    auto = None
    if xch is not None and xmode == "auto" and xch.mode == "inline" and not dry:
        auto = {}
        for mode in ("inline", "async"):
            xch.mode = mode
            loop.steps(max(1, args.warmup))
            sync(dry)
            dist.barrier()
            ta = time.perf_counter()
            loop.steps(args.steps)
            sync(dry)
            dist.barrier()
            t = torch.tensor([time.perf_counter() - ta], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            auto[mode] = round(float(t.item()) / args.steps * 1e6, 2)
        xch.mode = min(auto, key=auto.get)
        loop.one_step(0)
        offsets_ok = offsets_ok and xch.verify(stream)
        loop.steps(max(1, args.warmup))

    if multi:
        dist.barrier()
    sync(dry)
    # HIP events on the launch stream bracket the same K steps (GPU time of the timed loop): the
    # per-kernel durations are this time split by the kernels' ratio (measure_kernels), so they sum to
    # at most ms_per_step
    # No HIP events inside the timed region (default): the loop's GPU time comes from the same K steps
    # run again right after it, untimed, between two events.  r5i (profiles/r5i_timed_events.md): the
    # two event records cost ~0.3 us per step at the driver's 20 steps (graph 772-778 against 779-784
    # GiB/s).  RLE_BENCH_TIMED_EVENTS=1: the events bracket the timed steps themselves (round 4).
    timed_ev = os.environ.get("RLE_BENCH_TIMED_EVENTS", "0") != "0"
    ev = None if (dry or not timed_ev) else (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    if ev:
        ev[0].record(stream)
    loop.steps(args.steps)
    if ev:
        ev[1].record(stream)
    sync(dry)
    if multi:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    loop_gpu_s = ev[0].elapsed_time(ev[1]) * 1e-3 if ev else None
    if not dry and not timed_ev:
        loop.steps(max(1, args.warmup))
        sync(dry)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        loop.steps(args.steps)
        e1.record(stream)
        sync(dry)
        loop_gpu_s = e0.elapsed_time(e1) * 1e-3
    if multi:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        okt = torch.tensor([1 if ok else 0, 1 if offsets_ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = None if dry else bool(okt[0].item())
        offsets_ok = bool(okt[1].item())
        ut = torch.tensor([u_local], dtype=torch.int64, device=dev)
        dist.all_reduce(ut, op=dist.ReduceOp.SUM)
        total_u = int(ut.item())
    else:
        total_u = u_local

    # the same K steps in the other issue form, right after the timed loop (one rank): replayed from
    # one HIP graph when the headline issued them eagerly, or eagerly when it replayed a graph
    # (VERDICT r4 item 7, r5 item 3), so the launch share is visible beside the headline
    other = None
    if xch is None and not dry:
        was_plain = loop.plain
        try:
            if not was_plain:
                loop.capture_plain(args.steps)
                if args.warmup != args.steps:
                    loop.capture_plain(max(1, args.warmup))
            loop.plain = not was_plain
            loop.steps(max(1, args.warmup))
            sync(dry)
            t1 = time.perf_counter()
            loop.steps(args.steps)
            sync(dry)
            te = time.perf_counter() - t1
            other = {"value": round(total_u * args.steps / te / GIB, 3), "ms_per_step": round(te / args.steps * 1e3, 4)}
        except Exception as e:
            print(f"second issue form failed ({e})", file=sys.stderr)
        loop.plain = was_plain
        loop.graphs.clear()
    eager = other if loop.plain else None
    graphed = other if not loop.plain else None
    # the headline is the faster of the two issue forms of the same K steps (the
    # graph replay was ~2 % slower than eager issue on every round-5 box, ~1 % faster on others)
    primary = {"value": total_u * args.steps / elapsed / GIB, "ms_per_step": elapsed / args.steps * 1e3}
    use_other = other is not None and other["value"] > primary["value"]
    if use_other:
        elapsed = other["ms_per_step"] * 1e-3 * args.steps
    headline_graph = loop.plain != use_other

    kern = roofline = conc = north = cpu = None
    if not dry:
        kern, roofline = measure_kernels(B, args, stream, u_local, c_bytes, loop_gpu_s,
                                         "timed_loop_events" if timed_ev else "rerun_events")
        if rank == 0 and not multi:
            conc = concurrent_streams(B, wl, args, stream, dev)
            if not args.no_north_star and args.workload != "dec64k":
                loop.B = B = None   # the codec batch's HBM is released before the dec64k batch
                torch.cuda.empty_cache()
                north = north_star(args, stream, dev)
            cpu = cpu_leg(wl, args, c_bytes)

    if rank == 0:
        value = other["value"] if use_other else total_u * args.steps / elapsed / GIB
        par = f"shard round-robin over {world} GPU(s)"
        if xch is not None:
            par += {"inline": ", RCCL all-gather of sizes + scan, one library call per step on the codec stream",
                    "async": ", RCCL all-gather of sizes + scan per step on a side stream beside the codec "
                             "(one library call per step)",
                    "graph": ", RCCL all-gather of sizes + scan per step on a graph branch beside the codec "
                             "(whole timed loop captured in one HIP graph)",
                    "torch": ", all-gather of sizes via torch.distributed (" + ("gloo" if dry else "nccl") + ")"}[xch.mode]
        out = {"metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "u8",
               "data": "synthetic" if not dry else "dry run: no codec launches, closed-form sizes (CPU, gloo)",
               "config": {"workload": wl["desc"], "buffers_per_gpu": wl["n"],
                          "buffer_bytes": wl["size"] or "mixed 4 KiB-2 MiB",
                          "u_bytes_per_gpu": total_u // world, "c_bytes_rank0": c_bytes, "parallelism": par},
               "verified_bit_exact_roundtrip": ok, "host_wait": sched,
               "issue": ("one HIP graph of the K timed steps (captured before the timed region), replayed"
                         if headline_graph else "eager: 2 launches per step from the host")
                        + " (the faster of the two issue forms, each timed over the same K steps)",
               "timed_region_events": timed_ev,
               "value_eager": eager["value"] if eager else (round(primary["value"], 3) if not loop.plain else None),
               "ms_per_step_eager": eager["ms_per_step"] if eager else (round(primary["ms_per_step"], 4) if not loop.plain else None),
               "value_graph": graphed["value"] if graphed else (round(primary["value"], 3) if loop.plain else None),
               "ms_per_step_graph": graphed["ms_per_step"] if graphed else (round(primary["ms_per_step"], 4) if loop.plain else None),
               "kernels": kern, "roofline": roofline,
               "cpu_baseline": cpu, "north_star_dec64k": north, "concurrent_streams": conc}
        if xch is not None:
            out["exchange"] = {"mode": xch.mode, "offsets_match_process_group": offsets_ok, "graph_captured": graph_ok,
                               "error": str(xch.error) if xch.error else None, "default_mode_reason": XMODE_REASON,
                               "auto_us_per_step": auto}
        if dry:
            out["dry_run"] = True
        print(json.dumps(out), flush=True)
    if xch is not None:
        loop.graphs.clear()
        xch.close()
    if multi:
        dist.destroy_process_group()


def measure_kernels(B, args, stream, u_local, c_bytes, loop_gpu_s=None, loop_src="timed_loop_events"):
    """Per-kernel durations (HIP events on the launch stream; step_kernels), algorithmic bytes =
    U + C per launch, and the roofline object of the dominant kernel."""
    reps = max(10, min(args.steps, 50))
    t_enc, t_dec, detail = step_kernels(B, reps, stream, loop_gpu_s, args.steps, loop_src)
    alg = u_local + c_bytes
    # GBps: algorithmic bytes (U + C) per second, the roofline numerator; U_GiBps: uncompressed bytes
    # per second (SURVEY.md 8(d) reports both), also for the round trip
    kern = {"encode": {"us": t_enc * 1e6, "GBps": alg / t_enc / 1e9, "U_GiBps": u_local / t_enc / GIB},
            "decode": {"us": t_dec * 1e6, "GBps": alg / t_dec / 1e9, "U_GiBps": u_local / t_dec / GIB},
            "roundtrip": {"us": (t_enc + t_dec) * 1e6, "U_GiBps": u_local / (t_enc + t_dec) / GIB},
            "method": detail}
    dom = "encode" if t_enc >= t_dec else "decode"
    pmc = load_pmc(args.workload)
    traffic = pmc.get(dom) if isinstance(pmc, dict) else None
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(kern[dom]["GBps"], 2), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(kern[dom]["GBps"] / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "traffic_source": load_pmc("_source") if traffic is not None else None,
                "alg_bytes_per_launch": alg, "copy_ceiling": copy_ceiling(B, alg, reps, stream)}
    return kern, roofline


def concurrent_streams(B, wl, args, stream, dev):
    """Informational, not `value`: the same round trips with two batches in flight on two streams, as
    the drop-in runs when the server's worker threads (one HIP stream each) call it concurrently."""
    if B.u_bytes > (256 << 20) or args.steps <= 0 or args.no_concurrent:
        return None
    B2 = Batch(wl, 0, 1, dev)
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
    return conc


NS_ROUNDS = 5


def median(v):
    return sorted(v)[len(v) // 2]


def north_star(args, stream, dev):
    """The north-star figure: decode of 16384 x 64 KiB (zero / random / runs50 / runs90) as GB/s of
    (U + C) and as a fraction of 8 TB/s, beside the copy ceiling of the same bytes."""
    N = Batch(WORKLOADS["dec64k"], 0, 1, dev)
    N.encode(stream)
    N.calibrate()
    nc = int(N.clen.sum().item())
    # steady state: the first ~10 ms of run-heavy decode after an idle gap run ~10 % slower while the
    # shader clock ramps (profiles/r5al_pattern_rounds.jsonl: 463 us, then 409-416 us); so decode and
    # encode are timed in alternating rounds after one untimed round, and each reports its median
    dec, enc = (lambda: N.decode(stream)), (lambda: N.encode(stream))
    time_kernels(dec, 20, stream)
    tds, tes = [], []
    for _ in range(NS_ROUNDS):
        tds.append(time_kernels(dec, 20, stream))
        tes.append(time_kernels(enc, 20, stream))
    td, te = median(tds), median(tes)
    nok = bool(torch.equal(N.d_out, N.d_in))
    nalg = N.u_bytes + nc
    # the same memory traffic without the token work: one wave per buffer streaming its C bytes in
    # decode tiles and writing its U bytes, the decode's occupancy and issue order (overwrites d_out)
    pat = lambda: R.decode_pattern(N.d_c, N.coffs, N.clen, N.d_out, N.offs, N.lens, stream)
    tp = median([time_kernels(pat, 20, stream) for _ in range(NS_ROUNDS)])
    ncopy = copy_ceiling(N, nalg, 20, stream)
    north = {"workload": WORKLOADS["dec64k"]["desc"], "decode_us": td * 1e6,
             "decode_U_GiBps": N.u_bytes / td / GIB, "encode_U_GiBps": N.u_bytes / te / GIB,
             "decode_GBps": nalg / td / 1e9, "decode_frac": round(nalg / td / 1e9 / HBM_PEAK_GBPS, 4),
             "decode_frac_of_copy": round(ncopy["us"] / (td * 1e6), 4),
             "encode_GBps": nalg / te / 1e9, "u_bytes": N.u_bytes, "c_bytes": nc, "verified": nok,
             "copy_ceiling": ncopy,
             "pattern_ceiling": {"us": round(tp * 1e6, 3), "GBps": round(nalg / tp / 1e9, 2),
                                 "frac": round(nalg / tp / 1e9 / HBM_PEAK_GBPS, 4),
                                 "op": "rle_decode_pattern_device: the decode's tile reads and output writes, "
                                       "one wave per buffer, its occupancy and issue order, no token work"},
             "decode_frac_of_pattern": round(tp / td, 4),
             "timing": f"median of {NS_ROUNDS} rounds of 20 back-to-back launches after one untimed round",
             "decode_us_rounds": [round(t * 1e6, 1) for t in tds]}
    del N
    torch.cuda.empty_cache()
    return north


def cpu_leg(wl, args, c_bytes):
    if args.no_cpu:
        return None
    threads = min(16, os.cpu_count() or 1)
    r0 = cpu_baseline(wl, args.cpu_seconds, threads, "O0")
    r2 = cpu_baseline(wl, max(2.0, args.cpu_seconds / 2), threads, "O2")
    if not r0:
        return None
    return {"value": round(r0["rt_gibs"], 4), "unit": "GiB/s", "cores": threads, "kind": "reference",
            "sample": f"reference src/rleCompression.c compiled unchanged with its Makefile flags "
                      f"(-Wall -g -std=c99), {threads} pthreads, repeated passes over the same batch for "
                      f"{args.cpu_seconds:.0f} s ({r0['buffers']} buffers, {r0['u_bytes']} bytes)",
            "c_batch_match": r0["c_batch"] == c_bytes,
            "O2": round(r2["rt_gibs"], 4) if r2 else None}


def parse(argv=None):
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
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU / gloo rehearsal of the rank loop without codec launches (tests)")
    return ap.parse_args(argv)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; running {world} rank(s)", file=sys.stderr)
    run_rank(args)


if __name__ == "__main__":
    main()
