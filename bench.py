#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: device-resident Value-batch decode throughput on MI355X.

A "step" decodes one batch: a frame payload of From::Update(Id, F64) messages (configs[1],
10^7 records, 147,886,336 wire bytes), from HBM-resident wire bytes into HBM-resident id/f64
columns, through the C ABI. The K timed frames are a connection's backlog (nxg_decode_frames_async)
of 3 distinct frames decoded in rotation into 3 column sets, so that every decode streams from HBM
(3 x 308 MB is past three times the 256 MiB Infinity Cache). The frames' ids count up by one, so
the sequential-id decoder (nxg_decode_f64_seq.hip, one launch per frame) takes them; the
length-run decoder of any f64 frame (NXG_F64_PATH=run) and the same-frame rate of earlier rounds
are reported beside it. With --gpus N each rank decodes its own 10^7-record shard; the ids are
disjoint and there is no data-path collective ("weak" scaling). `value` is the whole-job
aggregate in M updates/s, over all ranks.

The inputs come from the product encoder (config 4). Outside the timed regions every leg is
checked once against the CPU oracle (oracle/nx_oracle.c, as the checker): decoded columns vs the
oracle's decode of the same wire bytes (every row and column), encoded bytes vs the oracle's
encode of the same columns. The oracle is also the cpu_baseline leg.

Also reported on the same JSON line:
  roofline       the decode's algorithmic bytes (W + 16 N) / mean time of one decode (HIP
                 events on the codec stream around the backlog) vs the 8 TB/s HBM3E peak;
  cpu_baseline   the C restatement of the reference decoder (oracle/, 1 core) on this host;
  extras         10^8-record decode (north-star size), mixed-tag decode (config 3), the
                 host-memory (PCIe-inclusive) decode path, f64 encode (config 4), subscriber
                 dispatch and publisher commit, the oracle on 16 host threads; with N>1, the
                 config-5 sharded encode + RCCL all-gather, the 10^8 batch decoded sharded by
                 record, mixed decode at 10^7 records per GPU (weak) and one 10^7-record mixed
                 frame decoded in N byte ranges (strong).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# the f64 decode (nxg_decode_f64_run.hip) of a stream of frames (nxg_decode_frames_async): one
# launch per frame, nxg_f64r_fused_kernel = the emit of frame j (reads W, writes 16 N) + the
# record-length probe of frame j + 1 (reads ~1 line per 32 KiB tile); the first frame's probe and
# the last frame's emit are launched alone. One call per frame (nxg_decode_updates_async) runs
# probe + emit as two launches.
KERNEL_DEC_F64 = "nxg_f64r_fused_kernel"
KERNELS_DEC_F64 = ["nxg_f64r_probe_kernel", "nxg_f64r_fused_kernel", "nxg_f64r_emit_kernel"]
# the sequential-id decoder (nxg_decode_f64_seq.hip): one launch per frame, the first choice for
# frames whose ids count up by one (a publisher updating all of its values)
KERNEL_SEQ = "nxg_f64s_kernel"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Rehearsal of the N > 1 path on a one-GPU box: BENCH_DIST_BACKEND=gloo BENCH_FORCE_DEVICE0=1
# runs every rank on cuda:0 with gloo collectives over host tensors (the driver's multi-GPU runs
# use RCCL, one GPU per rank).
BACKEND = os.environ.get("BENCH_DIST_BACKEND", "nccl")


def coll_device():
    return "cpu" if BACKEND == "gloo" else "cuda"


def dist_setup():
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("BENCH_FORCE_DEVICE0") == "1":
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if BACKEND == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world):
    from netidx_amd import shard
    return shard.max_over_ranks(x, world, device=coll_device())


def make_f64_wire(codec, n, rank):
    import netidx_amd
    from netidx_amd import synth
    ids, vals = synth.f64_columns(n, synth.SEED_F64, id_offset=rank * n)
    cols = netidx_amd.columns_from_arrays(ids, vals)
    wire = codec.encode_batch(cols)
    return cols, wire


# The GPU lowers its clocks while it idles (the host-side checks between legs take seconds): the
# first frames after an idle spell measured up to 8 % slower (scripts/exp_order.py). Every leg
# therefore runs its own operation for WARM_S seconds before its timed region.
WARM_S = 0.25
# time_decode's kernel-time pass: a spin kernel of this many GPU clock cycles (~0.2 ms) ahead of
# the first event (0: the wall-clock pass's events)
GATE_CYCLES = int(os.environ.get("BENCH_GATE_CYCLES", "500000"))


def warm(fn, sync, seconds=WARM_S):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        sync()


def time_decode(codec, wire, out, n, steps, warmup, world, stream, flags=0, stream_of_frames=False):
    """Returns (wall seconds max over ranks, mean ms per frame from HIP events, last status).
    `wire` / `out` may be lists: frame j is wire[j % len] decoded into out[j % len] (distinct
    frames and column sets: with 3 of them at 10^7 records the working set, 924 MB, is past three
    times the 256 MiB Infinity Cache, so every decode streams from HBM). stream_of_frames: the
    frames go through nxg_decode_frames_async (a connection's backlog), up to 500 per call; else
    one nxg_decode_updates_async per frame."""
    import torch
    wires = wire if isinstance(wire, (list, tuple)) else [wire]
    outs = out if isinstance(out, (list, tuple)) else [out]
    m_ = len(wires)

    def enqueue(k):
        if stream_of_frames:
            i = 0
            while i < k:
                m = min(500, k - i)
                sel = [(i + j) % m_ for j in range(m)]
                codec.decode_frames_async([wires[j].data_ptr() for j in sel],
                                          [wires[j].numel() for j in sel], [outs[j] for j in sel],
                                          flags)
                i += m
                if i < k:
                    codec.sync()
            return
        for i in range(k):
            j = i % m_
            codec.decode_async(wires[j].data_ptr(), wires[j].numel(), outs[j], flags)
            if (i + 1) % 500 == 0 and i + 1 < k:  # at most 512 async calls in flight
                codec.sync()

    for _ in range(warmup):
        enqueue(max(2, m_))
        codec.sync()
    warm(lambda: enqueue(max(2, m_)), codec.sync)
    barrier(world)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    enqueue(steps)
    e1.record(stream)
    st = codec.sync()
    torch.cuda.synchronize()
    barrier(world)
    wall = max_over_ranks(time.perf_counter() - t0, world)
    # The kernels' own time: the same frames again, the codec stream held by a short spin kernel
    # while the host enqueues them, so that the events do not count the GPU waiting for the
    # host's first submission (with the driver's --steps 20, ~50 us over 20 frames of 53 us)
    ms = e0.elapsed_time(e1) / steps
    if GATE_CYCLES:
        with torch.cuda.stream(stream):
            torch.cuda._sleep(GATE_CYCLES)
        e0.record(stream)
        enqueue(steps)
        e1.record(stream)
        st = codec.sync()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
    return wall, ms, st


def f64_kernel_name(codec):
    """The f64 decoder that produced the last decode: the sequential-id kernel or the
    length-run probe + emit (DevStatus.diag[1])."""
    return KERNEL_SEQ if codec.last_diag()[1] == 1 else " + ".join(KERNELS_DEC_F64)


def codec_run_path(device):
    """A second context whose f64 frames take the length-run decoder (NXG_F64_PATH=run)."""
    import netidx_amd
    os.environ["NXG_F64_PATH"] = "run"
    try:
        return netidx_amd.Codec(device)
    finally:
        del os.environ["NXG_F64_PATH"]


def _nxo():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import nxo
    return nxo


def oracle_check_decode(wire, cols, n, n_children=0, n_ctl=0):
    """Checker: the product's decoded columns (device) == the oracle's decode of the same wire
    bytes, every row and column. Returns the number of rows checked."""
    import numpy as np
    nxo = _nxo()
    w = wire.cpu().numpy() if hasattr(wire, "cpu") else wire
    o = nxo.decode(w, cap_rows=n + 1, cap_children=n_children + 1, cap_ctl=n_ctl + 1).trim()
    assert o["err_kind"] == 0 and len(o["id"]) == n, "oracle rejected the frame"
    g = cols.numpy()
    keys = ["id", "fixed"] if "aux" not in g else ["id", "tag", "fixed", "aux", "ctag", "cfixed",
                                                   "caux", "ctl_row", "ctl_off", "ctl_len",
                                                   "ctl_variant"]
    for k in keys:
        assert np.array_equal(g[k][: len(o[k])], o[k]) and len(g[k]) >= len(o[k]), \
            f"decode differs from the oracle in column {k}"
    if "aux" not in g:
        assert (o["tag"] == 9).all()
    return n


def oracle_check_encode(out_bytes, ids, vals=None, mixed=None):
    """Checker: the product's encoded bytes == the oracle encoder's bytes for the same columns."""
    import numpy as np
    nxo = _nxo()
    if mixed is None:
        ref = nxo.encode_f64(ids, vals)
    else:
        m = mixed
        n = len(m.id)
        d = nxo.Decoded(n, len(m.ctag) + 1, 1)
        for name in ("id", "tag", "fixed", "aux"):
            getattr(d, name)[:n] = getattr(m, name)
        d.ctag[:len(m.ctag)] = m.ctag
        d.cfixed[:len(m.ctag)] = m.cfixed
        d.caux[:len(m.ctag)] = m.caux
        d.s.n_rows, d.s.n_children, d.s.n_ctl = n, len(m.ctag), 0
        ref = np.frombuffer(nxo.encode(d, m.heap), np.uint8)
    got = out_bytes.cpu().numpy() if hasattr(out_bytes, "cpu") else out_bytes
    assert len(got) == len(ref) and np.array_equal(got, ref), "encode differs from the oracle"
    return len(ref)


def oracle_check_archive(buf, cols, m):
    """Checker for the archive legs: the product's encoded batch == the oracle encoder's bytes for
    the same columns, and the product's decode == the oracle's decode, every column."""
    import numpy as np
    nxo = _nxo()
    n = len(m.id)
    d = nxo.Decoded(n, len(m.ctag) + 1, 1)
    for name in ("id", "tag", "fixed", "aux"):
        getattr(d, name)[:n] = getattr(m, name)
    d.ctag[:len(m.ctag)] = m.ctag
    d.cfixed[:len(m.ctag)] = m.cfixed
    d.caux[:len(m.ctag)] = m.caux
    d.s.n_rows, d.s.n_children = n, len(m.ctag)
    ref = np.frombuffer(nxo.encode_archive(d, m.heap), np.uint8)
    got = buf.cpu().numpy()
    assert np.array_equal(got, ref), "archive encode differs from the oracle"
    o, used = nxo.decode_archive(got, cap_rows=n + 1, cap_children=len(m.ctag) + 1)
    o = o.trim()
    assert o["err_kind"] == 0 and used == len(got)
    g = cols.numpy()
    for k in ("id", "tag", "fixed", "aux", "ctag", "cfixed", "caux"):
        assert np.array_equal(g[k][: len(o[k])], o[k]), f"archive decode differs in {k}"
    return n


def host_cpu():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count()


def cpu_baseline(wire_host, n, seconds):
    """The oracle (C restatement of the reference's sequential decoder) on one host core."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import nxo
    reps, t_total = 0, 0.0
    while t_total < seconds or reps == 0:
        t0 = time.perf_counter()
        d = nxo.decode(wire_host, cap_rows=n + 1, cap_children=1, cap_ctl=1)
        t_total += time.perf_counter() - t0
        reps += 1
        assert d.s.err_kind == 0 and d.s.n_rows == n
    return n * reps / t_total, reps, t_total


def cpu_baseline_threads(wire_host, ids, seconds, threads=16):
    """Upper bound the reference does not reach: the oracle on `threads` host
    threads, the frame pre-cut at record boundaries (known from the ids: an f64 record is
    11 + varint_len(id) bytes). ctypes releases the GIL around each oracle call."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import nxo
    vl = 1 + (ids >= 2**7) + (ids >= 2**14) + (ids >= 2**21) + (ids >= 2**28)
    ends = np.cumsum(11 + vl.astype(np.int64))
    n = len(ids)
    cuts = [0] + [int(ends[n * k // threads - 1]) for k in range(1, threads)] + [len(wire_host)]
    parts = [wire_host[cuts[k]:cuts[k + 1]] for k in range(threads)]
    counts = [int(np.searchsorted(ends, cuts[k + 1], "right") - np.searchsorted(ends, cuts[k], "right"))
              for k in range(threads)]

    def one(k):
        d = nxo.decode(parts[k], cap_rows=counts[k] + 1, cap_children=1, cap_ctl=1)
        assert d.s.err_kind == 0 and d.s.n_rows == counts[k]

    reps, t_total = 0, 0.0
    with ThreadPoolExecutor(threads) as ex:
        while t_total < seconds or reps == 0:
            t0 = time.perf_counter()
            list(ex.map(one, range(threads)))
            t_total += time.perf_counter() - t0
            reps += 1
    return n * reps / t_total, reps, t_total


# host threads for the all-cores CPU baselines: the GPU box's CPU share per GPU (the harness sets
# OMP_NUM_THREADS = 16 there; os.cpu_count() reports the whole host, 256 on the driver's boxes, most
# of it other GPUs' share), capped at what this host has
def cpu_threads():
    try:
        t = int(os.environ.get("OMP_NUM_THREADS", "16"))
    except ValueError:
        t = 16
    return max(1, min(t, os.cpu_count() or 1))


CPU_THREADS_WHY = ("the GPU box's CPU share per GPU (OMP_NUM_THREADS there); os.cpu_count() "
                   "counts the whole host's cores, most of them other GPUs' share")


def _timed_reps(fn, seconds):
    reps, t = 0, 0.0
    while t < seconds or reps == 0:
        t0 = time.perf_counter()
        fn()
        t += time.perf_counter() - t0
        reps += 1
    return reps, t


def _decoded_of(m, rows=None):
    """Oracle-shaped columns (nxo.Decoded) of a MixedColumns row share (children re-based)."""
    import numpy as np
    nxo = _nxo()
    r0, r1 = rows if rows else (0, len(m.id))
    n = r1 - r0
    tag = m.tag[r0:r1]
    arr = tag == 19
    if arr.any():
        c0 = int(m.fixed[r0:r1][arr][0])
        last = np.flatnonzero(arr)[-1]
        c1 = int(m.fixed[r0 + last]) + int(m.aux[r0 + last])
    else:
        c0 = c1 = 0
    d = nxo.Decoded(n, c1 - c0 + 1, 1)
    d.id[:n] = m.id[r0:r1]
    d.tag[:n] = tag
    d.fixed[:n] = m.fixed[r0:r1]
    d.fixed[:n][arr] -= np.uint64(c0)
    d.aux[:n] = m.aux[r0:r1]
    d.ctag[:c1 - c0] = m.ctag[c0:c1]
    d.cfixed[:c1 - c0] = m.cfixed[c0:c1]
    d.caux[:c1 - c0] = m.caux[c0:c1]
    d.s.n_rows, d.s.n_children, d.s.n_ctl = n, c1 - c0, 0
    return d


def cpu_baselines_mixed(m, wire_host, seconds=3.0):
    """Config 3 beside the device numbers (north_star): the oracle's sequential decoder
    (the reference's receive_batch_fn loop, channel.rs:504-521) and encoder (queue_send,
    channel.rs:177-202) on 1 core and on cpu_threads() threads over row shares (each share its
    own frame: the messages are independent). Bounded samples, outside every timed GPU region."""
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor
    nxo = _nxo()
    n = len(m.id)
    nc = len(m.ctag)
    d = nxo.Decoded(n + 1, nc + 1, 1)

    def dec1():
        nxo.lib().nxo_decode_frame(wire_host.ctypes.data, len(wire_host), C.byref(d.s))
        assert d.s.err_kind == 0 and d.s.n_rows == n
    reps, t = _timed_reps(dec1, seconds)
    out = {"decode_1_core": {"value": round(n * reps / t / 1e6, 3), "unit": "M updates/s",
                             "cores": 1, "kind": "port",
                             "sample": f"the whole {n}-record mixed frame decoded {reps}x "
                                       f"({t:.1f} s) by oracle/nx_oracle.c"}}
    full = _decoded_of(m)

    def enc1():
        ln = nxo.lib().nxo_encoded_len(C.byref(full.s), m.heap.ctypes.data)
        buf = enc1.buf
        assert nxo.lib().nxo_encode(C.byref(full.s), m.heap.ctypes.data, buf.ctypes.data, ln) == ln
    import numpy as np
    enc1.buf = np.empty(len(wire_host) + 64, np.uint8)
    reps, t = _timed_reps(enc1, seconds)
    out["encode_1_core"] = {"value": round(n * reps / t / 1e6, 3), "unit": "M updates/s",
                            "cores": 1, "kind": "port",
                            "sample": f"the whole {n}-row batch encoded {reps}x ({t:.1f} s) by "
                                      "oracle/nx_oracle.c (encoded_len + encode)"}
    T = cpu_threads()
    cuts = [n * k // T for k in range(T + 1)]
    shares = [_decoded_of(m, (cuts[k], cuts[k + 1])) for k in range(T)]
    frames = [np.frombuffer(nxo.encode(sh, m.heap), np.uint8) for sh in shares]
    assert sum(len(f) for f in frames) == len(wire_host)
    outs = [nxo.Decoded(cuts[k + 1] - cuts[k] + 1, sh.s.n_children + 1, 1)
            for k, sh in enumerate(shares)]
    bufs = [np.empty(len(f) + 64, np.uint8) for f in frames]

    def dec_k(k):
        nxo.lib().nxo_decode_frame(frames[k].ctypes.data, len(frames[k]), C.byref(outs[k].s))
        assert outs[k].s.err_kind == 0

    def enc_k(k):
        ln = nxo.lib().nxo_encoded_len(C.byref(shares[k].s), m.heap.ctypes.data)
        assert nxo.lib().nxo_encode(C.byref(shares[k].s), m.heap.ctypes.data,
                                    bufs[k].ctypes.data, ln) == ln
    with ThreadPoolExecutor(T) as ex:
        reps, t = _timed_reps(lambda: list(ex.map(dec_k, range(T))), seconds)
        out["decode_threads"] = {
            "value": round(n * reps / t / 1e6, 3), "unit": "M updates/s", "cores": T,
            "kind": "port", "why_this_many": CPU_THREADS_WHY,
            "sample": f"the batch as {T} row-share frames decoded on {T} threads, {reps}x "
                      f"({t:.1f} s) (an upper bound: the reference decodes a frame on one task)"}
        reps, t = _timed_reps(lambda: list(ex.map(enc_k, range(T))), seconds)
        out["encode_threads"] = {
            "value": round(n * reps / t / 1e6, 3), "unit": "M updates/s", "cores": T,
            "kind": "port", "why_this_many": CPU_THREADS_WHY,
            "sample": f"the batch as {T} row shares encoded on {T} threads, {reps}x ({t:.1f} s)"}
    return out


def cpu_baselines_encode_f64(ids, vals, seconds=3.0):
    """Config 4 beside the device number: the oracle's f64 encoder (handle_updates ->
    queue_send, server.rs:604-629) on 1 core and on cpu_threads() threads over row shares."""
    import ctypes as C
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    nxo = _nxo()
    n = len(ids)
    cap = 21 * n + 16
    buf = np.empty(cap, np.uint8)

    def enc1():
        assert nxo.lib().nxo_encode_f64(ids.ctypes.data, vals.ctypes.data, n, buf.ctypes.data,
                                        cap) > 0
    reps, t = _timed_reps(enc1, seconds)
    out = {"encode_1_core": {"value": round(n * reps / t / 1e6, 3), "unit": "M updates/s",
                             "cores": 1, "kind": "port",
                             "sample": f"the whole {n}-record batch encoded {reps}x ({t:.1f} s) "
                                       "by oracle/nx_oracle.c"}}
    T = cpu_threads()
    cuts = [n * k // T for k in range(T + 1)]

    def enc_k(k):
        a, b = cuts[k], cuts[k + 1]
        assert nxo.lib().nxo_encode_f64(ids[a:].ctypes.data, vals[a:].ctypes.data, b - a,
                                        buf[21 * a:].ctypes.data, 21 * (b - a) + 16) >= 0
    with ThreadPoolExecutor(T) as ex:
        reps, t = _timed_reps(lambda: list(ex.map(enc_k, range(T))), seconds)
    out["encode_threads"] = {
        "value": round(n * reps / t / 1e6, 3), "unit": "M updates/s", "cores": T, "kind": "port",
        "why_this_many": CPU_THREADS_WHY,
        "sample": f"the batch as {T} row shares encoded on {T} threads, {reps}x ({t:.1f} s)"}
    return out


def read_traffic(records, kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if it matches."""
    for f in ("pmc_dec_f64.json", "pmc_dec_f64_100000000.json"):
        try:
            j = json.load(open(os.path.join(ROOT, "profiles", f)))
            if j.get("records") == records and j.get("kernel") == kernel:
                return j.get("hbm_bytes_per_launch")
        except Exception:
            pass
    return None


def read_split(records):
    """Per-kernel average durations of the f64 decoders at this size, from the committed rocprofv3
    kernel trace (profiles/f64_kernel_split.json), if present."""
    p = os.path.join(ROOT, "profiles", "f64_kernel_split.json")
    try:
        j = json.load(open(p))
        return j.get(str(records))
    except Exception:
        return None


def zstd_cpu_baseline(src, recs, want, dict_bytes, seconds=3.0):
    """The reference's CPU path for compressed archive records: one host core decompressing each
    record's zstd frame with the archive's dictionary (zstd::bulk::Decompressor::with_dictionary +
    decompress_to_buffer, netidx-archive/src/logfile/reader.rs:243-244, 453-477), here the
    system libzstd through ctypes (the zstd 0.13 crate wraps libzstd 1.5; this image has 1.4.8).
    Each record is a u32 BE plain length, then the frame. Returns the cpu_baseline object, or the
    reason it could not run."""
    import ctypes as C
    import numpy as np
    try:
        Z = C.CDLL("libzstd.so.1")
    except OSError as e:
        return {"error": f"libzstd not loadable: {e}"}
    Z.ZSTD_createDCtx.restype = C.c_void_p
    Z.ZSTD_createDDict.restype = C.c_void_p
    Z.ZSTD_createDDict.argtypes = [C.c_void_p, C.c_size_t]
    Z.ZSTD_decompress_usingDDict.restype = C.c_size_t
    Z.ZSTD_decompress_usingDDict.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                             C.c_size_t, C.c_void_p]
    Z.ZSTD_isError.argtypes = [C.c_size_t]
    dctx = Z.ZSTD_createDCtx()
    db = C.create_string_buffer(bytes(dict_bytes), len(dict_bytes))
    ddict = Z.ZSTD_createDDict(db, len(dict_bytes))
    src = np.ascontiguousarray(src)
    cap = max(len(w) for w in want) + 64
    dst = np.empty(cap, np.uint8)
    base = src.ctypes.data
    reps, t, nbytes = 0, 0.0, 0
    ok = True
    while t < seconds or reps == 0:
        t0 = time.perf_counter()
        for (off, ln), w in zip(recs, want):
            r = Z.ZSTD_decompress_usingDDict(dctx, dst.ctypes.data, cap, base + off + 4, ln - 4,
                                             ddict)
            ok &= not Z.ZSTD_isError(r) and r == len(w)
            nbytes += len(w)
        t += time.perf_counter() - t0
        reps += 1
    ok &= bool(np.array_equal(dst[:len(want[-1])], want[-1]))
    return {"value": round(nbytes / t / 1e9, 3), "unit": "plain GB/s", "cores": 1,
            "kind": "dependency (libzstd, the library the reference calls)", "ok": bool(ok),
            "sample": f"the {len(recs)} records decompressed {reps}x ({t:.1f} s) by the system "
                      "libzstd (ZSTD_decompress_usingDDict, one core)"}


def extras_single_gpu(codec, stream, steps, warmup):
    import netidx_amd
    import numpy as np
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    ex = {}
    # (a) north-star size: 10^8 f64 records on one GPU. Two frames and column sets in rotation
    # (3.1 GB each: far past the Infinity Cache either way), as one backlog; then the length-run
    # decoder on the same frames, and one call per frame.
    try:
        n = 100_000_000
        cols, wire = make_f64_wire(codec, n, 0)
        wires = [wire, wire.clone()]
        outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(2)]
        k = max(12, steps // 2)
        _, kms, st = time_decode(codec, wires, outs, n, k, 2, 1, stream, stream_of_frames=True)
        assert st.path == 1 and st.n_rows == n
        kname = f64_kernel_name(codec)
        _, kms1, st1 = time_decode(codec, wires, outs, n, k, 1, 1, stream)
        assert st1.path == 1 and st1.n_rows == n
        crun = codec_run_path(0)
        crun.set_stream(stream.cuda_stream)
        _, kms_run, st2 = time_decode(crun, wires, outs, n, k, 2, 1, stream, stream_of_frames=True)
        assert st2.path == 1 and st2.n_rows == n
        _, kms_run1, st3 = time_decode(crun, wires, outs, n, k, 1, 1, stream)
        assert st3.path == 1 and st3.n_rows == n
        crun.close()
        b = wire.numel() + 16 * n

        def fr(ms):
            return round(b / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)

        ex["decode_f64_1e8"] = {"records": n, "wire_bytes": wire.numel(),
                                "M_updates_s": round(n / (kms / 1e3) / 1e6, 1),
                                "kernel_ms": round(kms, 4), "hbm_frac": fr(kms),
                                "kernel": kname,
                                "timed": f"{k} frames as one backlog (nxg_decode_frames_async), 2 "
                                         "frames and column sets in rotation, HIP events on the "
                                         "codec stream",
                                "per_call_kernel_ms": round(kms1, 4), "per_call_hbm_frac": fr(kms1),
                                "length_run_decoder": {
                                    "kernels": " / ".join(KERNELS_DEC_F64),
                                    "backlog_kernel_ms": round(kms_run, 4),
                                    "backlog_hbm_frac": fr(kms_run),
                                    "per_call_kernel_ms": round(kms_run1, 4),
                                    "per_call_hbm_frac": fr(kms_run1)},
                                "kernel_split": read_split(n),
                                "traffic": read_traffic(n, kname),
                                "traffic_source": "profiles/pmc_dec_f64_100000000.json (FETCH_SIZE "
                                                  "x2 + WRITE_SIZE per launch, committed)",
                                "oracle_rows_checked": sum(oracle_check_decode(wire, o, n)
                                                           for o in outs)}
        del cols, wire, wires, outs
        torch.cuda.empty_cache()
    except Exception as e:  # report, never hide
        ex["decode_f64_1e8"] = {"error": repr(e)}
    # (a2) the same f64 batches with ids in random order (a batch updating an arbitrary subset of a
    # publisher's values, publisher/mod.rs:776-845): record lengths vary record to record, so the
    # length-run decoder hands the frames to the single-pass decoder (nxg_decode_f64_x.hip)
    for n in (10_000_000, 100_000_000):
        key = f"decode_f64_random_ids_{'1e7' if n == 10**7 else '1e8'}"
        try:
            ids, vals = synth.f64_columns(n, synth.SEED_F64)
            ids = np.random.default_rng(0x5EED0003).permutation(n).astype(np.uint64)
            cols = netidx_amd.columns_from_arrays(ids, vals)
            wire = codec.encode_batch(cols)
            out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
            k = max(6, steps // 4)
            wall, kms, st = time_decode(codec, wire, out, n, k, 2, 1, stream)
            assert st.path == 1 and st.n_rows == n
            b = wire.numel() + 16 * n
            ex[key] = {"records": n, "wire_bytes": wire.numel(),
                       "M_updates_s": round(n / (kms / 1e3) / 1e6, 1),
                       "kernel_ms": round(kms, 4),
                       "hbm_frac": round(b / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                       "kernel": "nxg_f64x_kernel (after the first frame: the length-run probe "
                                 "declines it, the next frames go straight to it)",
                       "oracle_rows_checked": oracle_check_decode(wire, out, n)}
            del cols, wire, out
            torch.cuda.empty_cache()
        except Exception as e:
            ex[key] = {"error": repr(e)}
    # (b) config 3: mixed-tag decode (general kernel)
    try:
        n = 10_000_000
        m = synth.mixed_columns(n)
        mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
        heap = torch.from_numpy(m.heap.copy()).cuda()
        wire = codec.encode_batch(mc, heap)
        out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
        wall, kms, st = time_decode(codec, wire, out, n, max(20, steps // 2), 2, 1, stream,
                                    flags=netidx_amd.HINT_MIXED)
        assert st.path == 4 and st.n_rows == n and st.err_kind == 0
        checked = oracle_check_decode(wire, out, n, len(m.ctag))
        nd = int((m.tag == 10).sum())
        ns = int((m.tag == 12).sum())
        na = int((m.tag == 19).sum())
        b = wire.numel() + n * (8 + 1 + 8 + 4) + 13 * len(m.ctag)
        ex["decode_mixed_1e7"] = {"records": n, "wire_bytes": wire.numel(),
                                  "M_updates_s": round(n / (kms / 1e3) / 1e6, 1),
                                  "kernel_ms": round(kms, 4),
                                  "hbm_frac": round(b / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                  "n_datetime": nd, "n_string": ns, "n_array": na,
                                  "n_children": len(m.ctag),
                                  "oracle_rows_checked": checked,
                                  "oracle_columns_checked": "all"}
        # the type-partitioned view of the decoded columns (nxg_partition_by_tag: per-tile LDS tag
        # histogram + scan, SURVEY 8a's optional output), checked against its numpy restatement
        try:
            view = codec.partition_by_tag(out)
            warm(lambda: codec.partition_by_tag(out, view), torch.cuda.synchronize)
            torch.cuda.synchronize()
            kp = max(3, steps // 4)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(kp):
                view = codec.partition_by_tag(out, view)
            e1.record(stream)
            torch.cuda.synchronize()
            pms = e0.elapsed_time(e1) / kp
            g = out.numpy()
            want = _nxo().partition_by_tag(g["tag"][:n], g["fixed"][:n], g["aux"][:n])
            got = view.numpy()
            assert all(np.array_equal(got[k], want[k]) for k in want), "partition differs"
            pb = n * (1 + 13 + 20)
            ex["partition_mixed_1e7"] = {
                "records": n, "call_ms": round(pms, 4),
                "M_rows_s": round(n / (pms / 1e3) / 1e6, 1),
                "hbm_frac": round(pb / (pms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes": pb,
                "kernels": "nxg_part_count / scan / offsets / place",
                "tags": {int(t): int(c) for t, c in enumerate(view.count) if c},
                "timed": "synchronous calls (host sync each), HIP events on the codec stream",
                "checked": "every array vs tests/nxo.py partition_by_tag (stable sort by tag)"}
            del view, g, want, got
        except Exception as e:
            ex["partition_mixed_1e7"] = {"error": repr(e)}
        # the mixed encode of the same columns (nxg_enc_rows_kernel), byte-identical to the wire
        dout = torch.empty(wire.numel() + 64, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            codec.encode_async(mc, heap, dout.data_ptr(), dout.numel())
            codec.sync()
        warm(lambda: codec.encode_async(mc, heap, dout.data_ptr(), dout.numel()), codec.sync)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        k = max(3, steps // 4)
        e0.record(stream)
        for _ in range(k):
            codec.encode_async(mc, heap, dout.data_ptr(), dout.numel())
        e1.record(stream)
        codec.sync()
        torch.cuda.synchronize()
        ems = e0.elapsed_time(e1) / k
        eb = oracle_check_encode(dout[: wire.numel()], None, mixed=m)
        text = int(m.aux[m.tag == 12].sum())  # string bytes copied from the heap
        be = wire.numel() + n * (8 + 1 + 8 + 4) + 13 * len(m.ctag) + text
        ex["encode_mixed_1e7"] = {"records": n, "wire_bytes": wire.numel(),
                                  "M_updates_s": round(n / (ems / 1e3) / 1e6, 1),
                                  "kernel_ms": round(ems, 4),
                                  "hbm_frac": round(be / (ems / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                  "oracle_bytes_checked": eb}
        try:
            cb = cpu_baselines_mixed(m, wire.cpu().numpy())
            ex["decode_mixed_1e7"]["cpu_baseline"] = cb["decode_1_core"]
            ex["decode_mixed_1e7"]["cpu_baseline_threads"] = cb["decode_threads"]
            ex["encode_mixed_1e7"]["cpu_baseline"] = cb["encode_1_core"]
            ex["encode_mixed_1e7"]["cpu_baseline_threads"] = cb["encode_threads"]
        except Exception as e:
            ex["decode_mixed_1e7"]["cpu_baseline"] = {"error": repr(e)}
        del mc, heap, wire, out, dout
        torch.cuda.empty_cache()
    except Exception as e:
        ex["decode_mixed_1e7"] = {"error": repr(e)}
    # (b0) config 3 as a live subscriber sees it: 1 % Heartbeats between the rows and 1 % of
    # the rows 200-byte strings (two-byte length prefixes), still on the fast mixed decoder
    try:
        n = 10_000_000
        m, cr, co, cl, cv = synth.mixed_columns_ctl(n)
        mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux,
                                            cr, co, cl, cv)
        heap = torch.from_numpy(m.heap.copy()).cuda()
        wire = codec.encode_batch(mc, heap)
        out = Columns(n + 1, len(m.ctag) + 1, len(cr) + 1, netidx_amd.LAYOUT_MIXED, "cuda")
        wall, kms, st = time_decode(codec, wire, out, n, max(20, steps // 2), 2, 1, stream,
                                    flags=netidx_amd.HINT_MIXED)
        assert st.path == 4 and st.n_rows == n and st.err_kind == 0, st
        assert st.n_heartbeat == len(cr)
        checked = oracle_check_decode(wire, out, n, len(m.ctag), len(cr))
        b = wire.numel() + n * (8 + 1 + 8 + 4) + 13 * len(m.ctag) + 21 * len(cr)
        ex["decode_mixed_ctl_1e7"] = {
            "records": n, "wire_bytes": wire.numel(), "n_heartbeat": len(cr),
            "n_long_string": int((m.aux[m.tag == 12] >= 100).sum()), "path": st.path,
            "M_updates_s": round(n / (kms / 1e3) / 1e6, 1), "kernel_ms": round(kms, 4),
            "hbm_frac": round(b / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "oracle_rows_checked": checked, "oracle_columns_checked": "all (ctl included)"}
        del mc, heap, wire, out
        torch.cuda.empty_cache()
    except Exception as e:
        ex["decode_mixed_ctl_1e7"] = {"error": repr(e)}
    # (b1) archive batches (Vec<BatchItem>): 10^7 items of the config-3 value
    # mix with 5 % Event::Unsubscribed; the product encoder writes the batch, the product decoder
    # reads it back; both checked once against the oracle. Wall clock per synchronous call.
    try:
        n = 10_000_000
        m = synth.archive_columns(n)
        mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
        heap = torch.from_numpy(m.heap.copy()).cuda()
        buf = codec.encode_archive(mc, heap)
        out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
        k = max(3, steps // 4)
        for _ in range(2):
            codec.encode_archive(mc, heap, buf)
            st, used = codec.decode_archive(buf, buf.numel(), out)
        warm(lambda: codec.decode_archive(buf, buf.numel(), out), torch.cuda.synchronize)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            codec.encode_archive(mc, heap, buf)
        torch.cuda.synchronize()
        t_enc = (time.perf_counter() - t0) / k
        t0 = time.perf_counter()
        for _ in range(k):
            st, used = codec.decode_archive(buf, buf.numel(), out)
        torch.cuda.synchronize()
        t_dec = (time.perf_counter() - t0) / k
        assert st.n_rows == n and used == buf.numel()
        checked = oracle_check_archive(buf, out, m)
        b = buf.numel() + n * (8 + 1 + 8 + 4) + 13 * len(m.ctag)
        # cpu_baseline: the reference reads an archive batch on one host core (reader.rs:449-477,
        # Pack decode of the Vec<BatchItem>): the oracle's decode_archive, 1 core, a bounded
        # sample (the whole batch, repeated for about 3 s)
        host_buf = buf.cpu().numpy()
        nxo = _nxo()
        reps, t_cpu = 0, 0.0
        while t_cpu < 3.0 or reps == 0:
            t0 = time.perf_counter()
            o, used_o = nxo.decode_archive(host_buf, cap_rows=n + 1, cap_children=len(m.ctag) + 1)
            t_cpu += time.perf_counter() - t0
            reps += 1
            assert used_o == len(host_buf)
        del o
        ex["archive_1e7"] = {"items": n, "batch_bytes": buf.numel(),
                             "decode_path": {5: "fast (nxg_fa_*)", 3: "exact (nxg_arch_*)"}.get(
                                 st.path, st.path),
                             "decode_ms": round(t_dec * 1e3, 3),
                             "decode_M_items_s": round(n / t_dec / 1e6, 1),
                             "decode_hbm_frac": round(b / t_dec / 1e9 / HBM_PEAK_GBS, 4),
                             "encode_ms": round(t_enc * 1e3, 3),
                             "encode_M_items_s": round(n / t_enc / 1e6, 1),
                             "oracle_items_checked": checked,
                             "cpu_baseline": {"value": round(n * reps / t_cpu / 1e6, 3),
                                              "unit": "M items/s", "cores": 1, "kind": "port",
                                              "sample": f"the whole {n}-item batch decoded "
                                                        f"{reps}x ({t_cpu:.1f} s) by "
                                                        "oracle/nx_oracle.c decode_archive"}}
        del mc, heap, buf, out
        torch.cuda.empty_cache()
    except Exception as e:
        ex["archive_1e7"] = {"error": repr(e)}
    # (b1z) compressed archive records (reader.rs:453-477): the committed libzstd fixtures'
    # dictionary records (level 19, the archive's trained dictionary; tests/golden/make_zstd.py),
    # repeated to ~100 MB of batches, decompressed on the GPU in one call (host records in, H2D
    # included, wall clock) and every output byte checked against the fixtures' plain bytes
    try:
        import json as _json
        gold = os.path.join(ROOT, "tests", "golden")
        man = _json.load(open(os.path.join(gold, "zstd_manifest.json")))
        rec = np.fromfile(os.path.join(gold, "zstd_records.bin"), np.uint8)
        plain = np.fromfile(os.path.join(gold, "zstd_plain.bin"), np.uint8)
        zdict = codec.zstd_dict(open(os.path.join(gold, "zstd_dict.bin"), "rb").read())
        es = [e for e in man["records"] if e["dict"] and not e["indexed"] and e["plain_len"]]
        per = sum(e["plain_len"] for e in es)
        R = max(1, (100 << 20) // per)
        parts, recs, want = [], [], []
        off = 0
        for _ in range(R):
            for e in es:
                parts.append(rec[e["rec_off"]:e["rec_off"] + e["rec_len"]])
                recs.append((off, e["rec_len"]))
                want.append(plain[e["plain_off"]:e["plain_off"] + e["plain_len"]])
                off += e["rec_len"]
        src = np.concatenate(parts)
        out, res = codec.archive_decompress(src, recs, False, zdict)
        k = max(3, steps // 40)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            out, res = codec.archive_decompress(src, recs, False, zdict, out=out)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / k
        host = out.cpu().numpy()
        assert all(r[2] == 0 for r in res), "a record failed to decompress"
        assert all(np.array_equal(host[r[0]:r[0] + r[1]], w) for r, w in zip(res, want)), \
            "decompressed bytes differ from the fixtures"
        tot = sum(r[1] for r in res)
        ex["archive_zstd_decompress"] = {
            "records": len(recs), "compressed_bytes": int(len(src)), "plain_bytes": int(tot),
            "ms": round(dt * 1e3, 3), "plain_GB_s": round(tot / dt / 1e9, 2),
            "note": "wall clock of nxg_archive_decompress from host records (H2D included); "
                    "libzstd fixtures (dictionary, level 19) repeated; every byte checked",
            "cpu_baseline": zstd_cpu_baseline(src, recs, want,
                                              open(os.path.join(gold, "zstd_dict.bin"), "rb").read())}
        zdict.close()
        del out
        torch.cuda.empty_cache()
    except Exception as e:
        ex["archive_zstd_decompress"] = {"error": repr(e)}
    # (b2) the socket-buffer path: host (pinned) frame -> device decode -> host (pinned) columns,
    # through the same synchronous call (nxg_decode_updates stages H2D and D2H itself); wall
    # clock, so PCIe Gen5 transfers are included. Never the bench `value`.
    try:
        n = 10_000_000
        cols, wire = make_f64_wire(codec, n, 0)
        hframe = wire.cpu().pin_memory()
        hout = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cpu")
        for _ in range(2):
            codec.decode_into(hframe, hframe.numel(), hout)
        k = max(3, steps // 4)
        t0 = time.perf_counter()
        for _ in range(k):
            st = codec.decode_into(hframe, hframe.numel(), hout)
        dt = (time.perf_counter() - t0) / k
        assert st.path == 1 and st.n_rows == n
        assert torch.equal(hout.fixed[:n], cols.fixed[:n].cpu())
        ex["decode_f64_1e7_host_pcie"] = {
            "records": n, "M_updates_s": round(n / dt / 1e6, 1), "ms": round(dt * 1e3, 3),
            "host_bytes_moved": wire.numel() + 16 * n,
            "GB_s_host_to_host": round((wire.numel() + 16 * n) / dt / 1e9, 2)}
        del cols, wire, hframe, hout
    except Exception as e:
        ex["decode_f64_1e7_host_pcie"] = {"error": repr(e)}
    # (b3) the same socket-buffer path for a stream of frames (a connection's read_task hands
    # over frame after frame, channel.rs:379-443): two contexts, each on its own stream, take
    # alternate frames; frame j's H2D and decode overlap frame j-1's D2H (PCIe is full duplex).
    # Wall clock per frame over F frames. Never the bench `value`.
    try:
        n = 10_000_000
        cols, wire = make_f64_wire(codec, n, 0)
        hframe = wire.cpu().pin_memory()
        W = wire.numel()
        ctxs, streams, dins, douts, hid, hval = [], [], [], [], [], []
        for k in range(2):
            c = netidx_amd.Codec(0)
            s = torch.cuda.Stream()
            c.set_stream(s.cuda_stream)
            ctxs.append(c)
            streams.append(s)
            dins.append(torch.empty(W, dtype=torch.uint8, device="cuda"))
            douts.append(Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda"))
            hid.append(torch.empty(n, dtype=torch.int64).pin_memory())
            hval.append(torch.empty(n, dtype=torch.int64).pin_memory())

        def enqueue_in(j):
            k = j % 2
            with torch.cuda.stream(streams[k]):
                dins[k].copy_(hframe, non_blocking=True)
            ctxs[k].decode_async(dins[k].data_ptr(), W, douts[k])

        def finish(j):
            k = j % 2
            st = ctxs[k].sync()
            assert st.path == 1 and st.n_rows == n
            with torch.cuda.stream(streams[k]):
                hid[k].copy_(douts[k].id[: st.n_rows], non_blocking=True)
                hval[k].copy_(douts[k].fixed[: st.n_rows], non_blocking=True)

        def run(frames):
            for j in range(frames):
                enqueue_in(j)
                if j > 0:
                    finish(j - 1)
            finish(frames - 1)
            for s in streams:
                s.synchronize()

        run(2)
        F = max(6, steps // 2)
        t0 = time.perf_counter()
        run(F)
        dt = (time.perf_counter() - t0) / F
        for k in range(2):
            assert torch.equal(hval[k], cols.fixed[:n].cpu()) and torch.equal(hid[k], cols.id[:n].cpu())
        ex["decode_f64_1e7_host_pipelined"] = {
            "records": n, "frames": F, "M_updates_s": round(n / dt / 1e6, 1),
            "ms_per_frame": round(dt * 1e3, 3),
            "GB_s_host_to_host": round((W + 16 * n) / dt / 1e9, 2)}
        for c in ctxs:
            c.close()
        del cols, wire, hframe, dins, douts, hid, hval
        torch.cuda.empty_cache()
    except Exception as e:
        ex["decode_f64_1e7_host_pipelined"] = {"error": repr(e)}
    # (b4) end to end through a loopback TCP socket, all in the library's C++ sessions
    # (nxg_session_*): handshake + To::Subscribe / From::Subscribed, then per frame the publisher
    # encodes on the GPU (nxg_encode_frames), copies to pinned memory and writes the frame; the
    # subscriber reads the socket into a pinned buffer, copies the frame to the device and
    # decodes it (device-resident columns). Wall clock per frame, F frames back to back.
    try:
        import threading
        n = 10_000_000
        cols, wire = make_f64_wire(codec, n, 0)
        W = wire.numel()
        F = 6
        pub = netidx_amd.Codec(0)
        dout = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        lst = netidx_amd.Session.listen()
        res = {}

        def publisher():
            try:
                s = lst.accept()
                netidx_amd.msg_parse(s.recv_frame(), to=True)
                s.send(netidx_amd.msg_subscribed("/local/bench/0", 0, 16))
                for _ in range(F):
                    s.publish(pub, cols)
                s.close()
            except Exception as e:
                res["err"] = repr(e)

        th = threading.Thread(target=publisher)
        th.start()
        sub = netidx_amd.Session.connect("127.0.0.1", lst.port)
        sub.send(netidx_amd.msg_subscribe("/local/bench/0"))
        netidx_amd.msg_parse(sub.recv_frame())
        sub.recv_decode(codec, dout)  # the first frame (buffers sized, pages touched)
        t0 = time.perf_counter()
        for _ in range(F - 1):
            st, flen = sub.recv_decode(codec, dout)
            assert st.path == 1 and st.n_rows == n and flen == W
        dt = (time.perf_counter() - t0) / (F - 1)
        th.join()
        sub.close()
        lst.close()
        pub.close()
        assert "err" not in res, res.get("err")
        assert torch.equal(dout.fixed[:n], cols.fixed[:n])
        ex["socket_e2e_f64_1e7"] = {
            "records": n, "frames": F - 1, "frame_bytes": W, "ms_per_frame": round(dt * 1e3, 2),
            "M_updates_s": round(n / dt / 1e6, 1), "GB_s_socket": round(W / dt / 1e9, 2),
            "path": "C++ sessions: GPU encode -> D2H pinned -> TCP loopback -> pinned recv -> "
                    "H2D -> GPU decode (device columns)"}
        del cols, wire, dout
        torch.cuda.empty_cache()
    except Exception as e:
        ex["socket_e2e_f64_1e7"] = {"error": repr(e)}
    # (c) config 4: f64 encode from device columns, byte-identical round trip. A context of its
    # own, as a publisher's connection has: the random-order legs above made this one's encodes
    # skip the sequential-id encoder for a while (it declined their batches)
    enc = None
    codec_main = codec
    try:
        n = 10_000_000
        enc = netidx_amd.Codec(0)
        enc.set_stream(stream.cuda_stream)
        codec = enc
        cols, wire = make_f64_wire(codec, n, 0)
        dout = torch.empty(wire.numel() + 64, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            codec.encode_async(cols, None, dout.data_ptr(), dout.numel())
            codec.sync()
        warm(lambda: codec.encode_async(cols, None, dout.data_ptr(), dout.numel()), codec.sync)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        k = max(3, steps // 2)
        e0.record(stream)
        for _ in range(k):
            codec.encode_async(cols, None, dout.data_ptr(), dout.numel())
        e1.record(stream)
        codec.sync()
        torch.cuda.synchronize()
        kms = e0.elapsed_time(e1) / k
        ids_h = cols.id[:n].cpu().numpy().view("uint64")
        vals_h = cols.fixed[:n].cpu().numpy().view("uint64")
        eb = oracle_check_encode(dout[: wire.numel()], ids_h, vals_h)
        b = wire.numel() + 16 * n
        ex["encode_f64_1e7"] = {"records": n, "M_updates_s": round(n / (kms / 1e3) / 1e6, 1),
                                "kernel_ms": round(kms, 4),
                                "hbm_frac": round(b / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                "kernel": ("nxg_enc_f64s_kernel (sequential ids)"
                                           if codec.last_encode_kernel() == "seq"
                                           else "nxg_enc_f64_kernel (tiled look-back)"),
                                "oracle_bytes_checked": eb}
        try:
            cb = cpu_baselines_encode_f64(ids_h, vals_h)
            ex["encode_f64_1e7"]["cpu_baseline"] = cb["encode_1_core"]
            ex["encode_f64_1e7"]["cpu_baseline_threads"] = cb["encode_threads"]
        except Exception as e:
            ex["encode_f64_1e7"]["cpu_baseline"] = {"error": repr(e)}
        del cols, wire, dout
        torch.cuda.empty_cache()
        # (c2) the north-star size: 10^8 records, 1.5 GB of wire
        try:
            n = 100_000_000
            ids_h, vals_h = synth.f64_columns(n, synth.SEED_F64)
            cols = netidx_amd.columns_from_arrays(ids_h, vals_h)
            W = codec.encoded_len(cols)
            dout = torch.empty(W + 64, dtype=torch.uint8, device="cuda")
            for _ in range(2):
                codec.encode_async(cols, None, dout.data_ptr(), dout.numel())
                codec.sync()
            warm(lambda: codec.encode_async(cols, None, dout.data_ptr(), dout.numel()), codec.sync)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            k = max(4, steps // 4)
            e0.record(stream)
            for _ in range(k):
                codec.encode_async(cols, None, dout.data_ptr(), dout.numel())
            e1.record(stream)
            codec.sync()
            torch.cuda.synchronize()
            kms = e0.elapsed_time(e1) / k
            eb = oracle_check_encode(dout[:W], ids_h, vals_h)
            b = W + 16 * n
            ex["encode_f64_1e8"] = {"records": n, "wire_bytes": W,
                                    "M_updates_s": round(n / (kms / 1e3) / 1e6, 1),
                                    "kernel_ms": round(kms, 4),
                                    "hbm_frac": round(b / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                    "kernel": ("nxg_enc_f64s_kernel (sequential ids)"
                                               if codec.last_encode_kernel() == "seq"
                                               else "nxg_enc_f64_kernel (tiled look-back)"),
                                    "timed": f"{k} async encodes of one column set into one "
                                             "buffer, HIP events on the codec stream",
                                    "oracle_bytes_checked": eb}
            del cols, dout
            torch.cuda.empty_cache()
        except Exception as e:
            ex["encode_f64_1e8"] = {"error": repr(e)}
    except Exception as e:
        ex["encode_f64_1e7"] = {"error": repr(e)}
    finally:
        codec = codec_main
        if enc is not None:
            enc.close()
    # (d) SURVEY 8f row 2: subscriber dispatch (process_updates_batch, connection.rs:546-567) of
    # 10^7 decoded updates: every id subscribed once, its stream on one of 16 channels, half of
    # the subscriptions keeping `last`. Checked against the oracle, which is also timed (1 core).
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import nxo
        n = 10_000_000
        n_chans = 16
        cols, wire = make_f64_wire(codec, n, 0)
        rng = np.random.default_rng(0x5EED0008)
        slot_of_id = np.arange(n, dtype=np.uint32)
        sub_id = rng.integers(0, 2**63, n, dtype=np.uint64)
        off = np.arange(n + 1, dtype=np.uint32)
        chan = rng.integers(0, n_chans, n, dtype=np.uint32)
        keep = (rng.random(n) < 0.5).astype(np.uint8)
        tab = netidx_amd.SubTable(slot_of_id, sub_id, off, chan, keep, n_chans)
        for _ in range(2):
            d = codec.dispatch_updates(tab, cols.id, n, cap=n)
        warm(lambda: codec.dispatch_updates(tab, cols.id, n, cap=n), torch.cuda.synchronize)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        k = max(3, steps // 4)
        e0.record(stream)
        for _ in range(k):
            d = codec.dispatch_updates(tab, cols.id, n, cap=n)
        e1.record(stream)
        torch.cuda.synchronize()
        kms = e0.elapsed_time(e1) / k
        ids_h = cols.id[:n].cpu().numpy().view(np.uint64)
        t0 = time.perf_counter()
        w = nxo.dispatch(ids_h, slot_of_id, sub_id, off, chan, keep, n_chans)
        cpu_s = time.perf_counter() - t0
        assert d.n_entries == n and np.array_equal(
            d.ent_row[:n].cpu().numpy().view(np.uint64), w[2])
        assert np.array_equal(d.ent_sub[:n].cpu().numpy().view(np.uint64), w[1])
        assert np.array_equal(d.last_row.cpu().numpy().view(np.uint64), w[3])
        n_last = int(keep.sum())
        # each row once: id, slot, stream offsets, channel, keep flag, SubId; entry written;
        # last row written for the kept subscriptions
        b = n * (8 + 4 + 8 + 4 + 1 + 8) + n * 16 + n_last * 8
        ex["dispatch_1e7"] = {"records": n, "channels": n_chans,
                              "M_updates_s": round(n / (kms / 1e3) / 1e6, 1),
                              "call_ms": round(kms, 4),
                              "hbm_frac": round(b / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                              "algorithmic_bytes": b,
                              "cpu_oracle_M_updates_s_1core": round(n / cpu_s / 1e6, 1)}
        del cols, wire, tab, d
        torch.cuda.empty_cache()
    except Exception as e:
        ex["dispatch_1e7"] = {"error": repr(e)}
    # (e) SURVEY 8a row a23: the publisher's commit (UpdateBatch::commit, publisher/mod.rs:
    # 776-845) of 10^7 queued f64 updates, each Id published once and subscribed by 1 or 2 of 16
    # clients; half the rows are UpdateChanged, half of those equal to the current value.
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import nxo
        n = 10_000_000
        n_cl = 16
        rng = np.random.default_rng(0x5EED0009)
        ids, vals = synth.f64_columns(n, synth.SEED_F64)
        fan = 1 + (rng.random(n) < 0.5).astype(np.int64)
        off = np.concatenate([[0], np.cumsum(fan)]).astype(np.uint32)
        first = rng.integers(0, n_cl, n)
        second = (first + 1 + rng.integers(0, n_cl - 1, n)) % n_cl
        client = np.empty(int(off[-1]), np.uint32)
        client[off[:-1]] = first
        two = fan == 2
        client[off[:-1][two] + 1] = second[two]
        kind = np.where(np.arange(n) % 2 == 0, 1, 0).astype(np.uint8)
        same = rng.random(n) < 0.5
        cur = np.where(same, vals, vals ^ np.uint64(1)).astype(np.uint64)
        slot_of_id = np.zeros(int(ids.max()) + 1, np.uint32)
        slot_of_id[ids] = np.arange(n, dtype=np.uint32)
        tab = netidx_amd.PubTable(slot_of_id, off, client, n_cl, None, cur)  # slot s = row s
        batch = netidx_amd.columns_from_arrays(ids, vals)
        dkind = torch.from_numpy(kind).cuda()
        cap = int(off[-1])
        for _ in range(2):
            d = codec.publish_commit(tab, batch, dkind, cap=cap)
        warm(lambda: codec.publish_commit(tab, batch, dkind, cap=cap), torch.cuda.synchronize)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        k = max(3, steps // 4)
        e0.record(stream)
        for _ in range(k):
            d = codec.publish_commit(tab, batch, dkind, cap=cap)
        e1.record(stream)
        torch.cuda.synchronize()
        kms = e0.elapsed_time(e1) / k
        t0 = time.perf_counter()
        w = nxo.publish_commit(ids, np.full(n, 9, np.uint8), vals, np.zeros(n, np.uint32),
                               np.zeros(1, np.uint8), kind, np.zeros(n, np.uint32), slot_of_id,
                               off, client, n_cl, np.full(n, 9, np.uint8), cur,
                               np.zeros(n, np.uint32), np.zeros(1, np.uint8))
        cpu_s = time.perf_counter() - t0
        assert d.n_entries == len(w[1])
        assert np.array_equal(d.ent_row[: d.n_entries].cpu().numpy().view(np.uint64), w[2])
        assert np.array_equal(d.last_row.cpu().numpy().view(np.uint64), w[3])
        # each row once: Id, value, kind, slot, client offsets, current value; entries written
        b = n * (8 + 8 + 1 + 4 + 8 + 8) + d.n_entries * (16 + 4) + n * 8
        ex["publish_commit_1e7"] = {"records": n, "clients": n_cl, "entries": int(d.n_entries),
                                    "M_updates_s": round(n / (kms / 1e3) / 1e6, 1),
                                    "call_ms": round(kms, 4),
                                    "hbm_frac": round(b / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                    "cpu_oracle_M_updates_s_1core": round(n / cpu_s / 1e6, 1)}
        del tab, batch, d
        torch.cuda.empty_cache()
    except Exception as e:
        ex["publish_commit_1e7"] = {"error": repr(e)}
    return ex


def make_comm(codec, world, rank, buffers):
    """The library's communicator for the multi-rank protocols (nxg_multi.cpp): RCCL
    (nxg_comm_init; its id broadcast over torch.distributed), or -- where RCCL cannot serve, gloo
    rehearsals with ranks sharing one GPU -- the same protocols over a torch.distributed transport
    (nxg_comm_init_ops, netidx_amd/shard.py gloo_comm; `buffers` are staged through the host)."""
    import netidx_amd
    import torch.distributed as dist
    from netidx_amd import shard
    if BACKEND == "gloo":
        return shard.gloo_comm(codec, world, rank, buffers)
    obj = [netidx_amd.Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return netidx_amd.Comm(codec, world, rank, obj[0])


def extras_multi_gpu(codec, world, rank, stream):
    """N > 1. Config 5: 10^8 records sharded by record; each rank encodes its shard straight
    into its place in the full frame and grouped send/recv over RCCL deliver every shard to every
    GPU (nxg_encode_allgather: one 8-byte all-gather of the sizes, no padding or copies). Then
    that one frame is decoded in N byte ranges, one per GPU (nxg_decode_sharded: each GPU takes
    the messages that start in its range, the ranges' summaries are all-gathered and linked),
    and config 3 (mixed) runs at 10^7 records per GPU (weak scaling). Times: the slowest rank's
    wall clock (barrier + device sync on both sides)."""
    import netidx_amd
    import numpy as np
    import torch
    from netidx_amd import shard, synth
    from netidx_amd.codec import Columns
    total = 100_000_000
    ex = {}
    # Each leg catches its own failure, after the leg's collectives (the library's protocols fail
    # on every rank at the same step; the checks run after the timing's all-reduce), so one
    # failing leg is reported and the ranks go on to the next leg together.
    comm = None
    dout = None
    W = 0
    b, e = shard.shard_range(total, world, rank)
    n = e - b
    via = ("rccl (nxg_encode_allgather)" if BACKEND != "gloo" else
           "gloo transport via nxg_comm_init_ops (nxg_encode_allgather)")
    try:
        ids, vals = synth.f64_columns(n, synth.SEED_8GPU, id_offset=b)
        cols = netidx_amd.columns_from_arrays(ids, vals)
        del ids, vals
        cap = 15 * total + 64
        dout = torch.empty(cap, dtype=torch.uint8, device="cuda")
        comm = make_comm(codec, world, rank, [dout])

        def encode_gather():
            return comm.encode_allgather(cols, None, dout.data_ptr(), cap)

        times = []
        for it in range(3):
            barrier(world)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            W, offs = encode_gather()
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        t = max_over_ranks(min(times), world)
        del cols
        # check: the frame's length is the whole batch's
        assert W == 1_497_886_336, W
        ex["encode_allgather_1e8"] = {"records": total, "wire_bytes": W, "world": world,
                                      "via": via, "encode_allgather_ms": round(t * 1e3, 3),
                                      "M_updates_s": round(total / t / 1e6, 1)}
    except Exception as err:
        ex["encode_allgather_1e8"] = {"error": repr(err)}
    # the one frame decoded in byte ranges (strong scaling)
    if comm is not None and W:
        try:
            out = Columns(n + 2 * total // world // 100 + 1024, 0, 0, netidx_amd.LAYOUT_F64, "cuda")

            def decode_ranges():
                return comm.decode_sharded(dout, W, out)

            decode_ranges()
            times = []
            for it in range(5):
                barrier(world)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                row_off, rng = decode_ranges()
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t0)
            t = max_over_ranks(min(times), world)
            nr = int(rng.n_rows)
            # checker: rows [row_off, row_off + nr) of the batch (ids are the global row numbers)
            got_id = out.id[:nr].cpu().numpy().view(np.uint64)
            got_val = out.fixed[:nr].cpu().numpy().view(np.uint64)
            assert np.array_equal(got_id, np.arange(row_off, row_off + nr, dtype=np.uint64))
            _, want_val = synth.f64_columns(nr, synth.SEED_8GPU, id_offset=row_off)
            assert np.array_equal(got_val, want_val), "range decode is not bit-exact"
            ex["decode_f64_1e8_byte_ranges"] = {
                "records": total, "world": world,
                "via": via.replace("nxg_encode_allgather", "nxg_decode_sharded"),
                "ms_slowest_rank": round(t * 1e3, 4), "M_updates_s": round(total / t / 1e6, 1)}
            del out
        except Exception as err:
            ex["decode_f64_1e8_byte_ranges"] = {"error": repr(err)}
    if comm is not None:
        comm.close()
    del dout
    torch.cuda.empty_cache()
    # config 3 per GPU (weak scaling): each rank decodes its own 10^7-record mixed batch
    nm = 10_000_000
    m = synth.mixed_columns(nm)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    wire = codec.encode_batch(mc, heap)
    try:
        out = Columns(nm + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
        wall, kms, st = time_decode(codec, wire, out, nm, 5, 1, world, stream,
                                    flags=netidx_amd.HINT_MIXED)
        kmax = max_over_ranks(kms, world)
        assert st.path == 4 and st.n_rows == nm and st.err_kind == 0, st
        # every column equals the encode input it was made from (the encoder is the oracle's,
        # checked byte for byte on rank 0 in the N=1 extras)
        nc = len(m.ctag)
        for k in ("id", "tag", "aux"):
            assert torch.equal(out.t[k][:nm], mc.t[k][:nm]), f"mixed decode differs in column {k}"
        for k in ("ctag", "cfixed", "caux"):
            assert torch.equal(out.t[k][:nc], mc.t[k][:nc]), f"mixed decode differs in column {k}"
        # fixed: the value for scalars; for text the frame offset of the bytes (the input's is a
        # heap offset), so the text itself is compared
        txt = out.tag[:nm] == 12
        assert torch.equal(out.fixed[:nm][~txt], mc.fixed[:nm][~txt]), "mixed decode differs in fixed"
        lens = out.aux[:nm][txt].long()
        rep = torch.repeat_interleave(torch.arange(len(lens), device=lens.device), lens)
        pos = torch.arange(int(lens.sum()), device=lens.device) - (torch.cumsum(lens, 0) - lens)[rep]
        assert torch.equal(wire[out.fixed[:nm][txt][rep] + pos], heap[mc.fixed[:nm][txt][rep] + pos]), \
            "mixed decode differs in text bytes"
        ex["decode_mixed_1e7_per_gpu"] = {
            "records_per_gpu": nm, "world": world, "kernel_ms_slowest_rank": round(kmax, 4),
            "M_updates_s": round(world * nm / (kmax / 1e3) / 1e6, 1)}
        del out
    except Exception as err:
        ex["decode_mixed_1e7_per_gpu"] = {"error": repr(err)}
    # config 3 strong-scaled: the SAME 10^7-record mixed frame (one connection's batch, as every
    # rank holds config 5's frame after the all-gather) decoded in N byte ranges, one per GPU
    # (nxg_decode_sharded: the fast mixed decoder in range mode, ranges linked)
    comm = None
    try:
        comm = make_comm(codec, world, rank, [wire])
        Wm = wire.numel()
        sout = Columns.for_frame(Wm // world + 65536, netidx_amd.LAYOUT_MIXED, "cuda")

        def decode_mixed_ranges():
            return comm.decode_sharded(wire, Wm, sout)

        decode_mixed_ranges()
        times = []
        for it in range(5):
            barrier(world)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            row_off, rng = decode_mixed_ranges()
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        t = max_over_ranks(min(times), world)
        check_mixed_range(wire, heap, mc, sout, row_off, rng, nm)
        ex["decode_mixed_1e7_byte_ranges"] = {
            "records": nm, "world": world, "wire_bytes": Wm, "range_path": int(rng.ok),
            "via": ("rccl" if BACKEND != "gloo" else "gloo transport via nxg_comm_init_ops") +
                   " (nxg_decode_sharded: fast mixed decoder in range mode)",
            "ms_slowest_rank": round(t * 1e3, 4), "M_updates_s": round(nm / t / 1e6, 1)}
    except Exception as err:
        ex["decode_mixed_1e7_byte_ranges"] = {"error": repr(err)}
    finally:
        if comm is not None:
            comm.close()
    return ex


def check_mixed_range(wire, heap, mc, out, row_off, rng, nm):
    """One rank's byte range of a mixed frame against the encode input it was made from: rows
    [row_off, row_off + n) of every column (array child indices from the range's first child,
    text compared byte for byte), and the children of those rows."""
    import torch
    n = int(rng.n_rows)
    assert rng.ok == 1 and row_off + n <= nm, (row_off, n, rng.ok)
    sl = slice(row_off, row_off + n)
    for k in ("id", "tag", "aux"):
        assert torch.equal(out.t[k][:n], mc.t[k][sl]), f"mixed range differs in column {k}"
    tag = out.tag[:n]
    arr, txt = tag == 19, tag == 12
    plain = ~(arr | txt)
    assert torch.equal(out.fixed[:n][plain], mc.fixed[sl][plain]), "mixed range differs in fixed"
    if bool(arr.any()):
        c0 = int(mc.fixed[sl][arr][0]) - int(out.fixed[:n][arr][0])
        assert torch.equal(out.fixed[:n][arr] + c0, mc.fixed[sl][arr])
        nc = int(out.s.n_children)
        for k in ("ctag", "cfixed", "caux"):
            assert torch.equal(out.t[k][:nc], mc.t[k][c0:c0 + nc]), f"range children differ: {k}"
    lens = out.aux[:n][txt].long()
    if len(lens):
        rep = torch.repeat_interleave(torch.arange(len(lens), device=lens.device), lens)
        pos = torch.arange(int(lens.sum()), device=lens.device) - (torch.cumsum(lens, 0) - lens)[rep]
        assert torch.equal(wire[out.fixed[:n][txt][rep] + pos],
                           heap[mc.fixed[sl][txt][rep] + pos]), "mixed range differs in text"


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-extras", action="store_true")
    args = ap.parse_args()

    import torch
    import netidx_amd
    from netidx_amd.codec import Columns

    world, rank, local = dist_setup()
    codec = netidx_amd.Codec(local)
    stream = torch.cuda.Stream()
    codec.set_stream(stream.cuda_stream)
    n = args.records

    cols, wire = make_f64_wire(codec, n, rank)
    nbytes = wire.numel()
    # three distinct frames and column sets, decoded in rotation: each decode streams from HBM
    # (working set 3 x (W + 16 N) = 924 MB at 10^7 records, past 3 x the 256 MiB Infinity Cache)
    wires = [wire, wire.clone(), wire.clone()]
    outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(3)]
    wall, kms, st = time_decode(codec, wires, outs, n, args.steps, args.warmup, world, stream,
                                stream_of_frames=True)
    assert st.err_kind == 0 and st.path == 1 and st.n_rows == n, st
    kname = f64_kernel_name(codec)
    # the same frame into the same columns every time (cache-assisted; earlier rounds' method)
    _, kms_same, st1 = time_decode(codec, wire, outs[0], n, max(20, args.steps // 4), 2, world,
                                   stream, stream_of_frames=True)
    assert st1.err_kind == 0 and st1.path == 1 and st1.n_rows == n, st1
    # one nxg_decode_updates_async per frame (no backlog), the same frames in rotation
    _, kms_call, st3 = time_decode(codec, wires, outs, n, max(20, args.steps // 4), 2, world,
                                   stream, stream_of_frames=False)
    assert st3.err_kind == 0 and st3.path == 1 and st3.n_rows == n, st3
    # the length-run decoder (any f64 frame; probe of frame j + 1 fused into the emit of frame j)
    crun = codec_run_path(local)
    crun.set_stream(stream.cuda_stream)
    _, kms_run, st2 = time_decode(crun, wires, outs, n, max(20, args.steps // 4), 2, world,
                                  stream, stream_of_frames=True)
    assert st2.err_kind == 0 and st2.path == 1 and st2.n_rows == n, st2
    crun.close()
    # checker, outside the timed regions: every row of every column set against the oracle's
    # decode of the same bytes
    checked = sum(oracle_check_decode(wire, o, n) for o in outs) if rank == 0 else 0

    value = world * n * args.steps / wall / 1e6
    alg_bytes = nbytes + 16 * n
    achieved = alg_bytes / (kms / 1e3) / 1e9

    def frac(ms):
        return round(alg_bytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)

    line = {
        "metric": "Value-batch decode: M updates/s/GPU + GiB/s (device-resident) vs HBM roofline",
        "value": round(value, 2),
        "unit": "M updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SplitMix64 f64 values, sequential ids; wire made by the product "
                "encoder); 3 distinct frames decoded in rotation into 3 column sets",
        "config": {"workload": "decode 10^7-record all-f64 From::Update batch per GPU "
                               "(BASELINE configs[1])",
                   "records_per_gpu": n, "wire_bytes_per_gpu": nbytes,
                   "parallelism": f"shard-per-gpu x{world} (no data-path collective)"},
        "per_gpu_M_updates_s": round(value / world, 2),
        "oracle_rows_checked": checked,
        "gib_per_s": round(world * alg_bytes * args.steps / wall / 2**30, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": read_traffic(n, kname),
                     "traffic_source": "profiles/pmc_dec_f64.json (rocprofv3 FETCH_SIZE x2 + "
                                       "WRITE_SIZE per decode, committed; not measured in this run)",
                     "kernel": kname,
                     "kernel_ms": round(kms, 4), "algorithmic_bytes_per_launch": alg_bytes,
                     "timed": "HIP events on the codec stream around the whole backlog of frames "
                              "(nxg_decode_frames_async), divided by the frames; 3 distinct "
                              "frames and column sets in rotation (every decode from HBM); a "
                              "second pass of the same frames after the wall-clock one, the "
                              f"stream held by a {GATE_CYCLES}-cycle spin kernel while the host "
                              "enqueues them (the events count no wait for the first submission)"},
        "method": "stream of frames: a connection's backlog through nxg_decode_frames_async "
                  "(round 3 on); per_call: one nxg_decode_updates_async per frame",
        "per_call": {"kernel_ms": round(kms_call, 4), "frac": frac(kms_call),
                     "timed": "one nxg_decode_updates_async per frame, the 3 frames in rotation, "
                              "HIP events on the codec stream"},
        "same_frame": {"kernel_ms": round(kms_same, 4), "frac": frac(kms_same),
                       "timed": "one frame into one column set every time (rounds 1-3's method: "
                                "partly served by the Infinity Cache)"},
        "length_run_decoder": {"kernel_ms": round(kms_run, 4), "frac": frac(kms_run),
                               "kernels": " / ".join(KERNELS_DEC_F64),
                               "timed": "NXG_F64_PATH=run: the decoder of any f64 frame, the 3 "
                                        "frames in rotation as one backlog"},
    }
    if rank == 0 and world == 1:
        host = wire.cpu().numpy()
        ups, reps, secs = cpu_baseline(host, n, args.cpu_seconds)
        model, nproc = host_cpu()
        line["cpu_baseline"] = {"value": round(ups / 1e6, 3), "unit": "M updates/s", "cores": 1,
                                "kind": "port", "cpu_model": model, "host_nproc": nproc,
                                "sample": f"full {n}-record f64 frame decoded {reps}x "
                                          f"({secs:.1f} s) by oracle/nx_oracle.c"}
        if not args.no_extras:
            line["extras"] = extras_single_gpu(codec, stream, min(args.steps, 40), args.warmup)
            T = cpu_threads()
            ups, reps, secs = cpu_baseline_threads(host, cols.id.cpu().numpy().view("uint64"),
                                                   min(args.cpu_seconds, 5.0), T)
            line["extras"]["cpu_baseline_threads"] = {
                "value": round(ups / 1e6, 3), "unit": "M updates/s", "cores": T,
                "kind": "port", "why_this_many": CPU_THREADS_WHY, "host_nproc": nproc,
                "sample": f"full {n}-record frame cut at record boundaries into {T} sub-frames, "
                          f"decoded {reps}x ({secs:.1f} s) by oracle/nx_oracle.c on {T} threads"}
    elif world > 1 and not args.no_extras:
        try:
            ex = extras_multi_gpu(codec, world, rank, stream)
        except Exception as e:  # report, never lose the line (each leg catches its own below)
            ex = {"error": repr(e)}
        if rank == 0:
            line["extras"] = ex
    if rank == 0:
        print(json.dumps(line), flush=True)
    codec.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
