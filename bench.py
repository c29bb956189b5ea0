"""Benchmark of the MI355X CTR forward hot path (BASELINE.json metric).

Default (N=1) workload — the configuration the metric is quoted on:
  DeepFM embedding-lookup + feature-interaction forward (the north-star hot
  path: ids -> 26 embedding rows -> x = [dense | emb] -> FMLayer logit), batch
  4096, 26 sparse fields x 1e7 rows, embedding dim 16 (one 16.64 GB fp32
  table), 13 dense features, FM k=10, int32 ids uniform per field, a pool of 64
  pre-generated batches rotated per step, inputs resident in HBM.  One step =
  one rs_embed_fm_fwd launch over one batch.

  N>1 (driver: torch.distributed.run, one rank per GPU) and --sharded at
  N=1: the SAME workload (26 x 1e7 x 16 table, embed + FM logit, 4096 local
  samples per rank: weak scaling) with the table row-sharded over the ranks
  (recommender_system_amd/sharded.py ShardedEmbeddingFM, pipelined partial
  protocol: per batch one RCCL all-to-all of [row ids | FM partials] records
  + one rs_shard_fm_pipe launch).  value = N*4096 / max-over-ranks step
  time; its roofline is the pipe kernel's (per-rank algorithmic bytes, the
  exchange records listed separately).  BASELINE config 5 (the DeepFM
  forward on a 1e8-row table, row-sharded, RCCL all-to-all of row ids and of
  rows, then the fused DeepFM kernel) is nested as `config5` (at N=1:
  `config5_n1`).

Also measured (nested in the JSON line, not `value`):
  * `roofline`: the fused gather+FM kernel's algorithmic bytes per launch
    (1,824 B/sample x 4096 + 18.9 KB of parameters) / its
    average launch duration from HIP events recorded around every timed launch
    on the launch stream; peak 8.0 TB/s.  `traffic` = PMC HBM bytes per launch
    from profiles/  or null.
  * `deepfm_forward`: the full DeepFM forward as ONE kernel (gather + FM +
    DNN 429-256-128-64-1 on fp32 MFMA + sigmoid head) samples/s.
  * `cpu_baseline`: the oracle's numpy fp32 restatement of the reference
    forward (TF unavailable) on the same table and batches, bounded sample.

Other configs (own JSON line): --config deepfm1e6 | dcn | din | pnn | nfm | afm | ffm | io | fm_train.
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM = 8.0e12
PEAK_F32 = 157.3e12
SEED = 20261015


def _dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.sharded:
        # RS_BENCH_BACKEND=gloo RS_BENCH_ONE_DEVICE=1: rehearsal of the N > 1
        # code path with every rank on device 0 (one-GPU box; gloo stages the
        # collectives through the host, so steps run eager) — never a result
        one_dev = os.environ.get("RS_BENCH_ONE_DEVICE") == "1"
        backend = os.environ.get("RS_BENCH_BACKEND", "nccl")
        torch.cuda.set_device(0 if one_dev else local)
        import torch.distributed as dist
        for key, val in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29533"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(key, val)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", 0 if one_dev else local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank


def _host_wait_mode(mode):
    """How the host waits for the device (hipSetDeviceFlags, before the device
    is first used; RS_BENCH_SYNC): 'spin' (the default) = busy-wait
    (hipDeviceScheduleSpin), as a latency-bound serving loop would set it;
    'default' = the runtime's own choice; 'yield' = hipDeviceScheduleYield.
    The synchronisations around the timed region return sooner: +3 % on the
    20-step line (profiles/r3_sync_mode_ab.jsonl)."""
    flags = {"": None, "default": None, "spin": 1, "yield": 2}[mode]
    if flags is None or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return  # multi-rank runs keep the runtime's default (the flag is per device, set before its first use)
    import ctypes
    with open("/proc/self/maps") as f:  # the HIP runtime torch loaded
        path = next(l.split()[-1] for l in f if "libamdhip64.so" in l)
    rc = ctypes.CDLL(path).hipSetDeviceFlags(ctypes.c_uint(flags))
    print(f"bench: hipSetDeviceFlags({flags}) -> {rc}", file=sys.stderr)


def _barrier(world):
    if world > 1 or _dist_on():
        import torch.distributed as dist
        dist.barrier()


def _dist_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def _max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _timed(fn, steps, warmup, world, events=True, begin=None, end=None):
    """Run warmup, then exactly `steps` timed steps between barrier+sync on
    both sides; returns (seconds, [per-step event ms]).  begin/end bracket
    multi-stream steps (their per-step events are then not kept)."""
    if begin is not None:
        begin()
        events = False
    for i in range(warmup):
        fn(i)
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    for i in range(steps):
        if events:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn(warmup + i)
            e.record()
            evs.append((s, e))
        else:
            fn(warmup + i)
    if end is not None:
        end()
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = [s.elapsed_time(e) for s, e in evs]
    return _max_over_ranks(dt, world), ms


def _capture(fn, first, count, begin=None, end=None):
    """HIP graph of `count` consecutive steps fn(first) .. fn(first+count-1);
    begin/end (optional) fork side streams off the capture stream and join
    them back (multi-stream steps)."""
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            if begin is not None:
                begin()
            for i in range(count):
                fn(first + i)
            if end is not None:
                end()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    return g


# nested legs (never a line's `value`) time at least this many steps: at the
# driver's --steps 20 a 10-step leg carried ~2-4 us per step of graph-launch
# and sync overhead (r4: deepfm_forward 24.1 us on the driver vs 22.0 at 200)
NESTED_MIN_STEPS = 128
# the peer legs' device waits: a working exchange waits microseconds; a broken
# one (e.g. mailbox visibility across GPUs of a node this code never ran on)
# gives up after ~1 s per wait instead of PeerExchange's default ~20 s, and
# the RCCL value stands
BENCH_PEER_SPIN = 1 << 20


def _timed_graph(fn, steps, warmup, world, chunk=64, begin=None, end=None):
    """Exactly `steps` steps replayed from HIP graphs of `chunk` steps (plus
    one tail graph), timed between barrier+sync; also returns the event time
    per graph launch-slot (kernel + inter-kernel boundary)."""
    if warmup:
        if begin is not None:
            begin()
        for i in range(warmup):
            fn(i)
        if end is not None:
            end()
    torch.cuda.synchronize()
    full, tail = divmod(steps, chunk)
    g_full = _capture(fn, 0, chunk, begin, end) if full else None
    g_tail = _capture(fn, 0, tail, begin, end) if tail else None
    for g in (g_full, g_tail):
        if g is not None:
            g.replay()
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record()
    for _ in range(full):
        g_full.replay()
    if g_tail is not None:
        g_tail.replay()
    e.record()
    torch.cuda.synchronize()
    _barrier(world)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return _max_over_ranks(dt, world), s.elapsed_time(e) / steps


def _timed_graph_streams(fn, steps, n_streams, world):
    """`steps` independent steps spread round-robin over `n_streams` parallel
    branches of ONE HIP graph (fork/join on events); returns seconds."""
    main = torch.cuda.current_stream()
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(main)
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g, stream=cap):
            for st in streams:
                st.wait_stream(cap)
            for i in range(steps):
                st = streams[i % n_streams]
                with torch.cuda.stream(st):
                    fn(i)
            for st in streams:
                cap.wait_stream(st)
    main.wait_stream(cap)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    _barrier(world)
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    _barrier(world)
    return _max_over_ranks(time.perf_counter() - t0, world)


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _device_state():
    """Clocks, power and temperature of the GPU this rank runs on, read from
    sysfs in-process (no exec): the DRM card whose PCI address matches torch's
    current device.  `sclk` / `mclk` = the active DPM level (the line marked
    '*'); power in W, temperature in C.  Box-to-box spread in the numbers
     is read against these."""
    import glob
    st = {}
    try:
        p = torch.cuda.get_device_properties(torch.cuda.current_device())
        want = "%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0), p.pci_bus_id, p.pci_device_id)
    except Exception as e:  # noqa: BLE001 - the state is informative only
        return {"error": f"{type(e).__name__}: {e}"[:120]}
    for dev in sorted(glob.glob("/sys/class/drm/card[0-9]*/device")):
        if not os.path.basename(os.path.realpath(dev)).startswith(want):
            continue
        st["card"] = os.path.basename(os.path.dirname(dev))
        st["pci"] = os.path.basename(os.path.realpath(dev))
        for key, name in (("sclk", "pp_dpm_sclk"), ("mclk", "pp_dpm_mclk"), ("fclk", "pp_dpm_fclk")):
            txt = _read(os.path.join(dev, name))
            if txt:
                act = [l.split(":", 1)[1].replace("*", "").strip() for l in txt.splitlines() if "*" in l]
                st[key] = act[0] if act else None
                st[key + "_levels"] = len(txt.splitlines())
        st["perf_level"] = _read(os.path.join(dev, "power_dpm_force_performance_level"))
        st["busy_percent"] = _read(os.path.join(dev, "gpu_busy_percent"))
        for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
            for key, name, scale in (("power_cap_W", "power1_cap", 1e-6), ("power_avg_W", "power1_average", 1e-6),
                                     ("power_W", "power1_input", 1e-6), ("sclk_MHz", "freq1_input", 1e-6),
                                     ("mclk_MHz", "freq2_input", 1e-6), ("temp_edge_C", "temp1_input", 1e-3),
                                     ("temp_hotspot_C", "temp2_input", 1e-3), ("temp_mem_C", "temp3_input", 1e-3)):
                v = _read(os.path.join(hw, name))
                if v is not None:
                    try:
                        st[key] = round(int(v) * scale, 1)
                    except ValueError:
                        pass
        break
    if not st:
        st["note"] = f"no /sys/class/drm card with PCI address {want}"
    return st


def _empty_kernel_slot(world):
    """Per-launch slot time of an empty 256 x 256 kernel replayed back to back
    from a hipGraph (dispatch + end of kernel + barrier: the box's floor under
    every graph-replayed step), in us."""
    from recommender_system_amd import _lib
    lib = _lib.lib()

    def step(i):
        _lib.check(lib.rs_diag_empty(256, 256, _lib.stream()), "rs_diag_empty")

    _, slot = _timed_graph(step, 256, 8, world, chunk=64)
    return round(slot * 1e3, 3)


def _pool(B, vocabs, nd, n_pool, device, dtype=torch.int32):
    g = torch.Generator(device=device)
    g.manual_seed(SEED)
    F = len(vocabs)
    ids = torch.empty(n_pool, B, F, dtype=dtype, device=device)
    for c, v in enumerate(vocabs):
        ids[:, :, c] = torch.randint(0, int(v), (n_pool, B), generator=g, device=device, dtype=dtype)
    dense = torch.rand(n_pool, B, nd, generator=g, device=device)
    return ids, dense


def _cpu_threads():
    try:
        from threadpoolctl import threadpool_info
        return max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
    except Exception:
        return 1


def cpu_baseline_hotpath(model, ids_pool, dense_pool, budget_s, max_batches=64):
    """Oracle (numpy fp32 op-for-op restatement of the reference forward) on the
    same table and batches: EmbedLayer + concat + FMLayer."""
    from oracle import ctr_oracle as O
    e = model.embed_layer
    t_copy = time.perf_counter()
    table = e.table.detach().cpu().numpy()
    t_copy = time.perf_counter() - t_copy
    tables = [table[o:o + v] for o, v in zip(e.row_offsets, e.vocab_sizes)]
    w0, w1, v = (p.detach().cpu().numpy() for p in (model.fm.w0, model.fm.w1, model.fm.v))
    n, t0 = 0, time.perf_counter()
    gpu_check = None
    while n < max_batches and (time.perf_counter() - t0) < budget_s:
        ids = ids_pool[n % ids_pool.shape[0]].cpu().numpy()
        dense = dense_pool[n % dense_pool.shape[0]].cpu().numpy()
        x = np.concatenate([dense, O.embed_layer(ids, tables, np.float32)], axis=-1)
        y = O.fm_layer(x, w0, w1, v, dt=np.float32)
        if gpu_check is None:
            gpu_check = (n, y)
        n += 1
    dt = time.perf_counter() - t0
    B = ids_pool.shape[1]
    return {"value": n * B / dt, "unit": "samples/s", "cores": _cpu_threads(), "kind": "port",
            "sample": f"{n} batches x {B} samples of the headline workload (same 1e7-row tables, "
                      f"numpy fp32 oracle = reference TF graph restated; TF not installed); "
                      f"table host copy {t_copy:.1f}s excluded"}, gpu_check


def _streamed_leg(args, world, model, ids_pool, dense_pool, step, logit, alg_bytes):
    """The hot path over S consecutive batch-B requests in ONE launch
    (DeepFM.fm_logit_stream / rs_embed_fm_fwd_hm_stream: tile g % tpb of batch
    g / tpb, the per-batch kernel's body): µs per batch, its HBM roofline
    fraction, and the check that every batch's logits are bit-identical to
    the single-launch step's.  min_blocks 1 / 2 (resident workgroups per CU)
    both timed; the faster is reported first."""
    B = ids_pool.shape[1]
    out = {}
    for S in (8, 32):
        sout = torch.empty(S, B, 1, device=ids_pool.device)
        ref = []
        for j in range(S):
            step(j)
            ref.append(logit.clone())
        legs = {}
        for mb in (1, 2):
            model.fm_logit_stream(dense_pool[:S], ids_pool[:S], min_blocks=mb, out=sout, check_ids=True)
            same = all(torch.equal(sout[j], ref[j]) for j in range(S))
            npool = ids_pool.shape[0] // S

            def stream_step(i, mb=mb):
                j0 = (i % npool) * S
                model.fm_logit_stream(dense_pool[j0:j0 + S], ids_pool[j0:j0 + S], min_blocks=mb, out=sout,
                                      check_ids=False)

            n = max(NESTED_MIN_STEPS // 4, args.steps // S)
            dt, slot = _timed_graph(stream_step, n, 5, world, chunk=8)
            us = slot * 1e3 / S
            legs[f"min_blocks_{mb}"] = {"us_per_batch": us, "launch_us": slot * 1e3,
                                        "samples_per_s": n * S * B / dt,
                                        "frac": alg_bytes / (us * 1e-6) / PEAK_HBM,
                                        "frac_of_random_row_ceiling": alg_bytes / (us * 1e-6) / 3.31e12,
                                        "bit_identical_to_single_launch": bool(same)}
        best = min(legs, key=lambda kk: legs[kk]["us_per_batch"])
        out[f"S{S}"] = dict(legs[best], best=best, **{"all": legs})
    out["note"] = ("one launch serves S consecutive batch-%d requests (ids/dense of batch s read from device memory "
                   "inside the kernel); us_per_batch = HIP-event slot of the graph-replayed launch / S; frac = the "
                   "headline's algorithmic bytes per batch / us_per_batch / 8 TB/s" % B)
    return out


def bench_hotpath(args, world, rank):
    import recommender_system_amd as rs
    from recommender_system_amd import _lib

    B, F, V, k, kfm, nd = args.batch, 26, int(args.vocab), 16, 10, 13
    vocabs = [V] * F
    dev = torch.device("cuda")
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    ids_pool, dense_pool = _pool(B, vocabs, nd, 64, dev)
    result = {}
    if world == 1 and not args.sharded:
        model = rs.DeepFM(cols, kfm, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=SEED, device=dev)
        e = model.embed_layer
        prep = model.fm.prepared(nd, F, k)
        logit = torch.empty(B, 1, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        lib = _lib.lib()
        tptr, optr, vptr = e.table.data_ptr(), e.field_offsets.data_ptr(), e.field_vocab.data_ptr()
        hoff, hvoc = e.host_meta()  # the field metadata also as kernel arguments (DeepFM.fm_logit's entry)
        pptr, w0ptr, lptr, eptr = prep.data_ptr(), model.fm.w0.data_ptr(), logit.data_ptr(), err.data_ptr()

        def step(i):
            j = i % ids_pool.shape[0]
            ids, dense = ids_pool[j], dense_pool[j]
            st = lib.rs_embed_fm_fwd_hm(ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, tptr, optr, vptr, hoff, hvoc,
                                        F, k, pptr, w0ptr, kfm, lptr, None, B, eptr, _lib.stream())
            if st:
                _lib.check(st, "rs_embed_fm_fwd_hm")

        # value: the K timed steps replayed from HIP graphs (no host launch cost)
        dt, slot_ms = _timed_graph(step, args.steps, args.warmup, world)
        # kernel duration: HIP events around each launch on the launch stream
        _, ms = _timed(step, args.steps, 0, world)
        assert int(err.item()) == 0
        kern_ms = slot_ms  # HIP events over the graph-replayed timed region, per launch
        bytes_per_launch = B * (F * 4 + nd * 4 + F * k * 4 + 4) + prep.numel() * 4
        alg_bytes = B * 1824 + 18880
        achieved = alg_bytes / (kern_ms * 1e-3)
        result["value"] = args.steps * B / dt
        result["ms_per_step"] = dt / args.steps * 1e3
        result["roofline"] = {"bound": "hbm", "achieved": achieved / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                              "frac": achieved / PEAK_HBM,
                              # the PMC file was measured on the 26 x 1e7 table: other vocabularies
                              # (--config deepfm1e6) have no pass of their own, so no traffic figure
                              "traffic": _pmc_traffic() if int(args.vocab) == int(1e7) else None,
                              "traffic_source": ("profiles/pmc_embed_fm.json (rocprofv3 PMC pass of this kernel at "
                                                 "this shape: TCC_EA0_RDREQ x 128 B + WRITE_SIZE per launch)"
                                                 if int(args.vocab) == int(1e7) else
                                                 "none: no PMC pass at this vocabulary"),
                              "kernel": "embed_fm_mfma_ka", "kernel_ms": kern_ms,
                              "kernel_ms_source": "HIP events around the graph-replayed timed region / steps "
                                                  "(kernel + back-to-back dispatch boundary)",
                              "eager_launch_event_ms_median": float(np.median(ms)),
                              "algorithmic_bytes_per_launch": alg_bytes,
                              "bytes_incl_packed_weights": int(bytes_per_launch),
                              "random_64B_row_ceiling_GBps": 3310.0,
                              "frac_of_random_row_ceiling": achieved / 3.31e12}
        # independent batches on parallel streams of one graph (secondary; the
        # headline value above is strictly sequential).  Each stream gets its
        # own output buffer.
        conc = {}
        for ns in (2, 4):
            logits = [torch.empty(B, 1, device=dev) for _ in range(ns)]

            def step_s(i, ns=ns, logits=logits):
                j = i % ids_pool.shape[0]
                ids, dense = ids_pool[j], dense_pool[j]
                st = lib.rs_embed_fm_fwd_hm(ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, tptr, optr, vptr, hoff,
                                            hvoc, F, k, pptr, w0ptr, kfm, logits[i % ns].data_ptr(), None, B, eptr,
                                            _lib.stream())
                if st:
                    _lib.check(st, "rs_embed_fm_fwd_hm")

            n = max(ns * 32, (args.steps // ns) * ns)
            t = _timed_graph_streams(step_s, n, ns, world)
            conc[f"{ns}_streams"] = {"samples_per_s": n * B / t, "us_per_batch": t / n * 1e6}
        result["concurrent_batches"] = conc
        # S consecutive batch requests served by ONE launch
        # (rs_embed_fm_fwd_hm_stream): the multi-batch floor of the same hot
        # path, nested (the value above stays one launch per batch)
        result["streamed"] = _streamed_leg(args, world, model, ids_pool, dense_pool, step, logit, alg_bytes)
        # secondary: Zipf(a=1.05) ids per field — repeated hot rows
        # hit L2 / the Infinity Cache, so this is cache-assisted, not the HBM line
        zrng = np.random.default_rng(SEED + 7)
        zipf_pool = torch.from_numpy(np.minimum(zrng.zipf(1.05, size=(16, B, F)) - 1, V - 1).astype(np.int32)).to(dev)
        zlogit = torch.empty(B, 1, device=dev)

        def step_z(i):
            ids, dense = zipf_pool[i % 16], dense_pool[i % 64]
            st = lib.rs_embed_fm_fwd_hm(ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, tptr, optr, vptr, hoff, hvoc,
                                        F, k, pptr, w0ptr, kfm, zlogit.data_ptr(), None, B, eptr, _lib.stream())
            if st:
                _lib.check(st, "rs_embed_fm_fwd_hm")

        dtz, slotz = _timed_graph(step_z, args.steps, args.warmup, world)
        uniq = float(np.mean([len(np.unique(zipf_pool[j].cpu().numpy())) for j in range(4)])) / (B * F)
        result["zipf_ids"] = {"samples_per_s": args.steps * B / dtz, "us_per_batch": slotz * 1e3,
                              "distinct_id_fraction": uniq,
                              "note": "Zipf(1.05) ids per field (clipped to the vocab), cache-assisted; the headline "
                                      "value is uniform ids"}
        # full DeepFM forward (secondary): one fused launch (gather + FM + DNN
        # tower + head), and the two-launch path (gather+FM emitting x, tower)
        xbuf = torch.empty(B, nd + F * k, device=dev)

        def full(i):
            j = i % ids_pool.shape[0]
            model.forward_fused((dense_pool[j], ids_pool[j]), check_ids=False)

        def two_launch(i):
            j = i % ids_pool.shape[0]
            fm = model.fm_logit((dense_pool[j], ids_pool[j]), x_out=xbuf, check_ids=False)
            model.dnn.tower(xbuf, extra=fm, c0=0.5, c1=0.5, head=True)

        n2 = max(NESTED_MIN_STEPS, args.steps // 5)
        # median of three timed runs: one host hiccup in a run of short graph
        # replays otherwise moves this nested number by ~10 % (r5: 22.3 vs 19.8)
        runs = sorted(_timed_graph(full, n2, args.warmup if r == 0 else 0, world, chunk=16) for r in range(3))
        dt2, slot2 = runs[1]
        dt3, _ = _timed_graph(two_launch, n2, args.warmup, world, chunk=16)
        flops = B * 2 * (429 * 256 + 256 * 128 + 128 * 64 + 64)
        result["deepfm_forward"] = {
            "samples_per_s": n2 * B / dt2, "ms_per_step": dt2 / n2 * 1e3, "slot_ms": slot2,
            "timing": f"median of 3 graph-replayed runs of {n2} steps (wall clock); slot_ms = HIP events per launch",
            "dnn_flop_per_step": flops,
            "dnn_tflops_incl_gather": flops / (dt2 / n2) / 1e12,
            "two_launch_samples_per_s": n2 * B / dt3,
            "note": "rs_deepfm_fwd: gather + FM + DNN 429-256-128-64-1 (fp32 MFMA, LDS-resident activations) + "
                    "sigmoid head in one launch; two_launch = rs_embed_fm_fwd emitting x + rs_mlp_fwd"}
        if args.cpu_baseline and rank == 0:
            cb, chk = cpu_baseline_hotpath(model, ids_pool, dense_pool, args.cpu_budget)
            j = chk[0]
            step(j)  # recompute batch j on the GPU for a cross-check
            torch.cuda.synchronize()
            g = logit.cpu().numpy()
            rms = float(np.sqrt(np.mean(chk[1] ** 2)))
            cb["max_scaled_diff_vs_gpu"] = float(np.max(np.abs(g - chk[1]) / np.maximum(np.abs(chk[1]), rms)))
            result["cpu_baseline"] = cb
        else:
            result["cpu_baseline"] = None
        # config 5 at world 1 with the exchange forced (RCCL self-exchange): the
        # same workload as the driver's N > 1 lines, so the 1 -> N curve has an anchor
        if not args.no_config5:
            _world1_group()
            c5, _ = bench_sharded_deepfm(args, 1, 0, lite=True)
            c5["note"] = ("BASELINE config 5 at N = 1: ShardedDeepFM forward on the 1e8-row table with the row "
                          "exchange forced through RCCL (self-exchange), B 4096 - the config5 field of the N > 1 "
                          "lines")
            result["config5_n1"] = c5
            # the N > 1 value's own protocol at world 1 (RCCL self-exchange):
            # what row-sharding costs on one GPU
            sfm, _, _ = bench_sharded_fm(args, 1, 0, vocabs, dense_pool, lite=True)
            sfm["note"] = ("the N > 1 value's protocol (row-sharded FM, pipelined partials) at world 1 with the "
                           "RCCL self-exchange forced - not what a world-1 job runs (it calls the unsharded "
                           "kernel, the value above)")
            result["fm_hotpath_sharded_n1"] = sfm
        # BASELINE configs 3 (DCN CrossNet) and 4 (DIN attention) under the
        # same clock: each its own line, nested (roofline + cpu_baseline)
        if not args.no_configs34:
            result["config3_n1"] = bench_dcn(args, 1, 0, nested=True)
            result["config4_n1"] = bench_din(args, 1, 0, nested=True)
    else:
        # N > 1 (and --sharded at N = 1): the metric's own workload, the
        # 26 x 1e7 table row-sharded over the ranks, B local samples per rank
        res, _, _ = bench_sharded_fm(args, world, rank, vocabs, dense_pool)
        result.update(res)
        result["value"] = res["samples_per_s"]
        # BASELINE config 5 (the DeepFM forward on the 1e8-row table) nested
        if not args.no_config5:
            c5, V5 = bench_sharded_deepfm(args, world, rank)
            c5["vocab_per_field"] = V5
            result["config5"] = c5
    return result


def _graph_capturable(fn, first, begin=None, end=None, count=1):
    """Capture (never replay) `count` steps in a HIP graph on every rank, then
    agree collectively: the RCCL all-to-alls are graph-captured only if every
    rank captured cleanly, otherwise every rank times the eager step."""
    import torch.distributed as dist
    if dist.get_backend() != "nccl":  # the gloo rehearsal: host-staged collectives cannot be captured
        return False, "gloo rehearsal (collectives staged through the host)"
    ok, why = 1, None
    try:
        _capture(fn, first, count, begin, end)
    except Exception as e:  # noqa: BLE001 - any capture failure selects the eager path
        ok, why = 0, f"{type(e).__name__}: {e}"[:200]
    torch.cuda.synchronize()
    t = torch.tensor([ok], dtype=torch.int32, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item()), why


def _peer_exchange_leg(args, world, sh, ids_pool, dense_pool, outs, rccl_step_ms, rccl_dt):
    """The pipelined sharded step with its all-to-all replaced by the
    peer-mapped exchange (sharded.PeerExchange / rs_peer_a2a: each rank
    writes its records straight into its peers' hipIpc-mapped mailboxes).
    First the same 8-batch stream through both exchanges, eager, from a fresh
    prologue: the logits must be bit-identical on every rank; then the timed
    steps (graph-replayed: the exchange has no host-side collective).  Any
    failure — setup, a device-side wait timeout, a mismatch — is collective
    and reported here; the RCCL numbers stand."""
    import torch.distributed as dist
    npool = ids_pool.shape[0]
    B = ids_pool.shape[1]
    T = 8
    seq = [(dense_pool[j % npool], ids_pool[j % npool]) for j in range(T)]
    try:
        ref = [o.clone() for o in sh.forward_stream(seq, check=True)]
        sh.use_peer_exchange(spin_limit=BENCH_PEER_SPIN)
        sh.forward_stream(seq[:1], check=True)  # one step first: a broken exchange fails after one bounded wait
        got = sh.forward_stream(seq, check=True)
        same = torch.tensor([int(all(torch.equal(a, b) for a, b in zip(ref, got)))], dtype=torch.int32,
                            device=ids_pool.device)
        if world > 1 or _dist_on():
            dist.all_reduce(same, op=dist.ReduceOp.MIN)
        identical = bool(same.item())
        sh.pipe_route(ids_pool[0])

        def pipelined(i):
            j, jp, jn = i % npool, (i - 1) % npool, (i + 1) % npool
            sh.pipe_step(prev=(dense_pool[jp], outs[(i - 1) % 2]), cur=ids_pool[j],
                         nxt=(dense_pool[jn], ids_pool[jn]))

        for i in range(args.warmup):
            pipelined(i)
        torch.cuda.synchronize()
        _barrier(world)
        dt, slot_ms = _timed_graph(pipelined, args.steps, 0, world, chunk=16)
        step_ms = _max_over_ranks(slot_ms, world)
        fl = torch.tensor([0], dtype=torch.int32, device=ids_pool.device)
        for ex in sh._peers.values():
            fl |= ex.err
        if world > 1 or _dist_on():
            dist.all_reduce(fl, op=dist.ReduceOp.MAX)
        if int(fl.item()):
            raise RuntimeError(f"peer exchange: device error flag {int(fl.item()):#x}")
        out = {"samples_per_s": world * args.steps * B / dt, "ms_per_step": dt / args.steps * 1e3,
               "slot_ms": step_ms, "timing": "HIP graph replay (peer exchange captured)",
               "bit_identical_to_rccl": identical,
               "faster_and_identical": identical and dt < rccl_dt,
               "rccl_ms_per_step": rccl_dt / args.steps * 1e3,
               "mailbox_bytes_per_rank": next(iter(sh._peers.values())).mbox_bytes,
               "note": "ONE launch per exchange (rs_peer_a2a): ready flag to every peer, 16-B stores of each "
                       "block into the peer's uncached mailbox, per-peer full flag, wait for every incoming "
                       "block; no RCCL"}
        out["two_deep"] = _two_deep_leg(args, world, sh, ids_pool, dense_pool, outs, ref, peer=True)
    except Exception as e:  # noqa: BLE001 — reported, the RCCL value stands
        out = {"error": repr(e)[:400]}
    finally:
        try:
            sh.close_peer_exchange()
        except Exception as e:  # noqa: BLE001
            out = dict(out, close_error=repr(e)[:200])
        sh.pipe_route(ids_pool[0])
    return out


def _two_deep_leg(args, world, sh, ids_pool, dense_pool, outs, ref, peer):
    """The TWO-DEEP pipelined step (sharded.py pipe2_step): the exchange of
    batch t+1 runs beside the pipe launch of batch t — inside it for the peer
    exchange (rs_shard_fm_pipe_peer, ONE launch per step), on the caller's
    stream beside a side-stream pipe launch for RCCL.  The same 8-batch stream
    as the one-deep RCCL reference first (bit-identity, collective), then
    graph-replayed timed steps.  Failures are reported; the caller keeps the
    other protocols' numbers."""
    import torch.distributed as dist
    npool = ids_pool.shape[0]
    B = ids_pool.shape[1]
    seq = [(dense_pool[j % npool], ids_pool[j % npool]) for j in range(len(ref))]
    try:
        sh.forward_stream2(seq[:1], check=True)  # one short stream first: a broken step fails fast
        got = sh.forward_stream2(seq, check=True)
        same = torch.tensor([int(all(torch.equal(a, b) for a, b in zip(ref, got)))], dtype=torch.int32,
                            device=ids_pool.device)
        if world > 1 or _dist_on():
            dist.all_reduce(same, op=dist.ReduceOp.MIN)
        identical = bool(same.item())
        sh.pipe2_prologue(ids_pool[0], ids_pool[1])

        def step(i):
            j = i % npool
            sh.pipe2_step(prev=(dense_pool[(i - 2) % npool], outs[i % 2]), cur=ids_pool[j],
                          nxt=ids_pool[(i + 2) % npool], exchange=True)

        begin, end = (None, None) if peer else (sh.pipe2_begin, sh.pipe2_join)
        sh.pipe2_begin()
        for i in range(args.warmup):
            step(i)
        sh.pipe2_join()
        torch.cuda.synchronize()
        _barrier(world)
        graphed, why = (True, None) if peer else _graph_capturable(step, 0, begin, end, count=2)
        steps = args.steps + args.steps % 2  # even: every graph keeps the slot parity of the stream
        if graphed:
            dt, slot_ms = _timed_graph(step, steps, 0, world, chunk=16, begin=begin, end=end)
            step_ms = _max_over_ranks(slot_ms, world)
        else:
            dt, ms = _timed(step, steps, 0, world, begin=begin, end=end)
            step_ms = _max_over_ranks(dt / steps * 1e3, world)
        fl = sh.ops.bad_flag()
        for ex in getattr(sh, "_peers", {}).values():
            fl |= ex.err
        if world > 1 or _dist_on():
            dist.all_reduce(fl, op=dist.ReduceOp.MAX)
        if int(fl.item()):
            raise RuntimeError(f"two-deep step: device error flag {int(fl.item()):#x}")
        return {"samples_per_s": world * steps * B / dt, "ms_per_step": dt / steps * 1e3,
                "slot_ms": step_ms, "steps": steps,
                "timing": ("HIP graph replay" if graphed else f"eager launches ({why})") +
                          (" (peer exchange inside the pipe launch)" if peer else " (RCCL + side-stream pipe)"),
                "bit_identical_to_rccl": identical,
                "protocol": ("two-deep: ONE launch per batch (rs_shard_fm_pipe_peer) = peer exchange of "
                             "[row ids of t+1 | partials of t-1] | combine t-2 | owner partials of t | route "
                             "t+2; two-slot mailboxes" if peer else
                             "two-deep: RCCL all-to-all of [row ids of t+1 | partials of t-1] on the step's "
                             "stream beside rs_shard_fm_pipe (combine t-2 | owner t | route t+2) on a side "
                             "stream; events order E(t+1) after P(t-1) and P(t) after E(t)")}
    except Exception as e:  # noqa: BLE001 — reported, the one-deep value stands
        return {"error": repr(e)[:400]}


def bench_sharded_fm(args, world, rank, vocabs, dense_pool, lite=False):
    """The headline workload (embedding lookup + FM logit, 26 x 1e7 x 16, B
    local samples per rank) with the table ROW-SHARDED over the ranks (weak
    scaling): the N > 1 line's `value`, and at N = 1 (forced RCCL
    self-exchange) the nested anchor `fm_hotpath_sharded_n1`.  Timed protocol
    (the value): owner-side FM partials, pipelined (sharded.py ``pipe_step``):
    per batch t ONE RCCL all-to-all carrying [row ids of t | FM partials of
    t-1], then ONE launch (rs_shard_fm_pipe) doing combine of t-1 | owner FM
    partials of t over its field range | field route of t+1.  Beside it: the
    pipe kernel alone (the roofline's kernel time), the unpipelined protocol
    (``forward``: two all-to-alls per batch) and, unless ``lite``, the
    cpu_baseline on rank 0; --extras adds the ROW exchange (``forward_slots``)
    and the data-parallel training step.  Steps are replayed from HIP graphs
    when RCCL capture works on every rank (decided collectively), eager
    otherwise."""
    if lite:  # nested (fm_hotpath_sharded_n1), not the line's value: at least NESTED_MIN_STEPS batches
        args = copy.copy(args)
        args.steps = max(args.steps, NESTED_MIN_STEPS)
    import torch.distributed as dist
    from recommender_system_amd.sharded import ShardedEmbeddingFM
    B, F, k = args.batch, len(vocabs), 16
    dev = torch.device("cuda")
    sh = ShardedEmbeddingFM(vocabs, k, 13, 10, device=dev, seed=SEED)
    sh._force_exchange = True
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + rank)
    ids_pool = torch.stack([torch.randint(0, vocabs[0], (B, F), generator=g, device=dev, dtype=torch.int32)
                            for _ in range(16)])
    out = torch.empty(B, 1, device=dev)
    outs = [torch.empty(B, 1, device=dev) for _ in range(2)]
    npool = ids_pool.shape[0]

    def pipelined(i):
        j, jp, jn = i % npool, (i - 1) % npool, (i + 1) % npool
        sh.pipe_step(prev=(dense_pool[jp], outs[(i - 1) % 2]), cur=ids_pool[j], nxt=(dense_pool[jn], ids_pool[jn]))

    def per_batch(fwd):
        def step(i):
            # fixed-size exchange, no host sync inside the step
            j = i % npool
            fwd(dense_pool[j], ids_pool[j], check=False, out=out)
        return step

    def run(step):
        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        _barrier(world)
        graphed, why = _graph_capturable(step, 0)
        if graphed:
            dt, slot_ms = _timed_graph(step, args.steps, 0, world, chunk=16)
            step_ms = _max_over_ranks(slot_ms, world)
        else:
            dt, ms = _timed(step, args.steps, 0, world)
            step_ms = _max_over_ranks(float(np.mean(ms)) if ms else dt / args.steps * 1e3, world)
        return dt, step_ms, ("HIP graph replay (RCCL captured)" if graphed else f"eager launches ({why})")

    sh.pipe_route(ids_pool[0])  # prologue of the stream: batch 0's row ids
    dt, step_ms, timing = run(pipelined)
    # the pipe kernel alone, on this rank's last received records (no
    # exchange: the same owner / route / combine work every launch)
    sb = sh._sbufs(B)

    def pipe_only(i):
        j = i % npool
        sh.ops.pipe(sh, sb["recv"], sb["send"], prev=(dense_pool[j], outs[0]), cur=ids_pool[j],
                    nxt=(dense_pool[j], ids_pool[j]))

    _, kslot = _timed_graph(pipe_only, args.steps, 2, world, chunk=16)
    kern_ms = _max_over_ranks(kslot, world)
    udt, ustep_ms, utiming = run(per_batch(sh.forward))
    f = sh.ops.bad_flag()  # any bad id during the timed steps?
    if world > 1 or _dist_on():
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
    if bool(f.item()):
        raise RuntimeError("sharded bench: bad ids during timing")
    # the two-deep step with the RCCL all-to-all (side-stream pipe launch)
    ref8 = [o.clone() for o in sh.forward_stream([(dense_pool[j], ids_pool[j]) for j in range(8)], check=True)]
    rccl2 = _two_deep_leg(args, world, sh, ids_pool, dense_pool, outs, ref8, peer=False)
    sh.pipe_route(ids_pool[0])
    peer = _peer_exchange_leg(args, world, sh, ids_pool, dense_pool, outs, step_ms, dt) \
        if os.environ.get("RS_BENCH_PEER", "1") != "0" else {"skipped": "RS_BENCH_PEER=0"}
    S, P = sh.slot_stride, sh.partial_width
    alg = B * 1824 + 18880
    rec_bytes = world * B * (S + P) * 4
    roof = {"bound": "hbm", "achieved": alg / (kern_ms * 1e-3) / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
            "frac": alg / (kern_ms * 1e-3) / PEAK_HBM, "traffic": None,
            "traffic_note": "no PMC pass on the driver's multi-GPU run; the N = 1 line's traffic is the unsharded "
                            "kernel's",
            "kernel": "shard_fm_pipe (rs_shard_fm_pipe: combine t-1 | owner FM partials of t | field route t+1)",
            "kernel_ms": kern_ms,
            "kernel_ms_source": "HIP events around graph-replayed launches of the pipe kernel alone on this rank's "
                                "received records (no exchange), max over ranks",
            "algorithmic_bytes_per_launch": alg,
            "algorithmic_bytes_note": "per rank and step: the headline's 1,824 B/sample (ids 104, dense 52, rows "
                                      "1,664, logit 4) x B local samples + 18,880 B of FM parameters - under uniform "
                                      "ids an owner reads B x F rows of 64 B on average; the exchange records are "
                                      "listed separately",
            "exchange_record_bytes_per_rank_each_way": rec_bytes,
            "record_bytes_per_launch": 2 * rec_bytes,
            "achieved_incl_records": (alg + 2 * rec_bytes) / (kern_ms * 1e-3) / 1e9,
            "step_ms": dt / args.steps * 1e3,
            "step_frac": alg / (dt / args.steps) / PEAK_HBM}
    res = {
        "samples_per_s": world * args.steps * B / dt, "ms_per_step": dt / args.steps * 1e3,
        "slot_ms": step_ms,
        "protocol": "owner-side FM partials, pipelined: ONE RCCL all-to-all of [row ids of t | FM partials of t-1] "
                    "records + ONE launch (combine t-1 | owner FM partials of t over its field range | field route "
                    "of t+1) per batch; fixed sizes, no host sync",
        "timing": timing, "roofline": roof, "lookups_per_rank": B * F, "rows_per_rank": sh.rows_per_rank,
        "owner_field_ranges": sh.owner_field_ranges, "bytes_per_rank_each_way": rec_bytes,
        "unpipelined": {"samples_per_s": world * args.steps * B / udt, "ms_per_step": udt / args.steps * 1e3,
                        "timing": utiming, "id_bytes_per_rank_each_way": world * B * S * 4,
                        "partial_bytes_per_rank_each_way": world * B * P * 4,
                        "note": "forward(): route, all-to-all ids, owner partials, all-to-all partials, combine"}}
    res["peer_exchange"] = peer
    res["rccl_two_deep"] = rccl2
    # every protocol moves the same records; the value is the fastest one whose
    # logits are bit-identical to the one-deep RCCL step's (all stay nested)
    res["rccl_pipelined"] = {"samples_per_s": res["samples_per_s"], "ms_per_step": res["ms_per_step"],
                             "slot_ms": res["slot_ms"], "timing": res["timing"]}
    cands = [("RCCL all_to_all (one-deep)", res["rccl_pipelined"], res["protocol"])]
    if peer.get("bit_identical_to_rccl"):
        cands.append(("peer-mapped mailboxes (rs_peer_a2a, one-deep)", peer,
                      res["protocol"].replace("ONE RCCL all-to-all", "ONE peer-mapped all-to-all (rs_peer_a2a)")))
    for name, leg in (("RCCL all_to_all (two-deep, side-stream pipe)", rccl2),
                      ("peer-mapped mailboxes inside the pipe launch (rs_shard_fm_pipe_peer, two-deep)",
                       peer.get("two_deep") or {})):
        if leg.get("bit_identical_to_rccl"):
            cands.append((name, leg, leg["protocol"]))
    name, best, proto = min(cands, key=lambda c: c[1]["ms_per_step"])
    res["samples_per_s"], res["ms_per_step"] = best["samples_per_s"], best["ms_per_step"]
    res["slot_ms"], res["timing"], res["protocol"] = best["slot_ms"], best["timing"], proto
    res["exchange"] = name
    res["exchange_candidates_ms_per_step"] = {c[0]: c[1]["ms_per_step"] for c in cands}
    if lite:
        return res, sh, ids_pool
    res["cpu_baseline"] = _cpu_leg_fm_sharded(args, world, rank, sh, dense_pool, ids_pool, B)
    if args.extras:
        # reference point: the same step with the row exchange
        rdt, _, rtiming = run(per_batch(sh.forward_slots))
        fl = sh.ops.flags(sh._bufs(B))
        dist.all_reduce(fl, op=dist.ReduceOp.MAX)
        bufs = sh._bufs(B)
        # data-parallel training step on the sharded table (sharded.py train_step)
        labels = (torch.rand(npool, B, generator=g, device=dev) < 0.25).to(torch.float32)

        def train(i):
            j = i % npool
            sh.train_step(dense_pool[j], ids_pool[j], labels[j], lr=0.01, check=False)

        tdt, _, ttiming = run(train)
        res["rows_protocol"] = {"samples_per_s": world * args.steps * B / rdt, "ms_per_step": rdt / args.steps * 1e3,
                                "timing": rtiming, "slots_per_peer": bufs["cap"],
                                "row_bytes_per_rank_each_way": world * bufs["cap"] * k * 4,
                                "overflow_during_timing": bool(fl[1].item()),
                                "note": "fixed-capacity row exchange (forward_slots): rows back to the requester"}
        res["train_step"] = {"samples_per_s": world * args.steps * B / tdt, "ms_per_step": tdt / args.steps * 1e3,
                             "timing": ttiming,
                             "note": "ShardedEmbeddingFM.train_step: partial-protocol forward (2 all-to-alls) + "
                                     "combine_grad, all-gather of [s | g] records, owner row grads + row-sparse SGD "
                                     "of the shard, all-reduce of the FM parameter grads, SGD + l2"}
    if world == 1:
        # the same pipelined step without the RCCL self-exchange (what a world-1
        # job runs: sharded.py skips the all-to-alls unless forced)
        sh._force_exchange = False
        sh.pipe_route(ids_pool[0])
        ldt, lstep_ms, ltiming = run(pipelined)
        sh._force_exchange = True
        res["world1_no_exchange"] = {
            "samples_per_s": args.steps * B / ldt, "ms_per_step": ldt / args.steps * 1e3, "slot_ms": lstep_ms,
            "timing": ltiming, "note": "world 1 without the self-exchange: rs_shard_fm_pipe alone per batch (the "
                                       "records alternate between two buffers); the RCCL lines above are the comparison"}
    return res, sh, ids_pool


def _cpu_leg_fm_sharded(args, world, rank, sh, dense_pool, ids_pool, B, n_batches=4):
    """cpu_baseline of the sharded headline line on rank 0: the oracle's numpy
    fp32 EmbedLayer + concat + FMLayer (layer/core.py:273-280,
    layer/interaction.py:106-114 restated; TF not installed) on rank 0's
    batches.  The rows come from the shards through the exact row exchange
    (``lookup``, collective), and the first batch's logits are compared with
    rank 0's GPU output of the same batch (``forward``, collective)."""
    if not args.cpu_baseline:
        return None
    out = torch.empty(B, 1, device=sh.device)
    host = []
    for j in range(n_batches):
        sh.forward(dense_pool[j], ids_pool[j], check=False, out=out)
        emb = sh.lookup(ids_pool[j])
        torch.cuda.synchronize()
        if rank == 0:
            host.append((dense_pool[j].cpu().numpy(), emb.reshape(B, -1).cpu().numpy(), out.cpu().numpy().copy()))
    _barrier(world)
    if rank != 0:
        return None
    from oracle import ctr_oracle as O
    w0, w1, v = (t.detach().cpu().numpy() for t in (sh.w0, sh.w1, sh.v))
    n, first, t0 = 0, None, time.perf_counter()
    while n < 64 and (time.perf_counter() - t0) < args.cpu_budget:
        dense, emb, gout = host[n % len(host)]
        y = O.fm_layer(np.concatenate([dense, emb], axis=-1), w0, w1, v, dt=np.float32)
        if first is None:
            first = (np.asarray(y, np.float64), gout)
        n += 1
    dt = time.perf_counter() - t0
    ref, gout = first
    rms = float(np.sqrt(np.mean(ref ** 2)))
    return {"value": n * B / dt, "unit": "samples/s", "cores": _cpu_threads(), "kind": "port",
            "sample": f"{n} batches x {B} samples of rank 0 (of {world}): numpy fp32 EmbedLayer + concat + FMLayer "
                      f"(the reference TF graph restated; TF not installed); the batch's rows copied from the "
                      f"shards through the exact row exchange",
            "max_scaled_diff_vs_gpu": float(np.max(np.abs(gout.reshape(ref.shape) - ref) /
                                                   np.maximum(np.abs(ref), rms)))}


def _cpu_leg_config5(args, world, rank, model, dense_pool, ids_pool, out, B, n_batches=4):
    """cpu_baseline of config 5 on rank 0: the oracle's numpy fp32 DeepFM
    (model/deepFM.py:23-31 restated; TF not installed) on rank 0's batches,
    with the embedding rows copied from the shards — every rank runs the
    sharded forward of those batches (the exchange is collective), rank 0 reads
    each lookup's row out of its row-exchange buffer (got[slot_of]) — and
    max_scaled_diff_vs_gpu against rank 0's GPU output of the same batch."""
    if not args.cpu_baseline:
        return None
    rb = model._rbufs(B, dedup=False)
    host = []
    for j in range(n_batches):
        model.forward((dense_pool[j], ids_pool[j]), check=False, out=out)
        torch.cuda.synchronize()
        if rank == 0:
            emb = rb["got"][rb["slot_of"].reshape(-1).long()].reshape(B, model.F, model.k)
            host.append((dense_pool[j].cpu().numpy(), emb.cpu().numpy(), out.cpu().numpy().copy()))
    _barrier(world)
    if rank != 0:
        return None
    from oracle import ctr_oracle as O
    c = lambda t: t.detach().cpu().numpy()
    p = {"w0": c(model.emb.w0), "w1": c(model.emb.w1), "v": c(model.emb.v),
         "dnn_hidden": [(c(l.kernel), c(l.bias)) for l in model.dnn.hidden_layer],
         "dnn_out": (c(model.dnn.output_layer.kernel), c(model.dnn.output_layer.bias))}
    ids = np.tile(np.arange(B, dtype=np.int64)[:, None], (1, model.F))
    n, first, t0 = 0, None, time.perf_counter()
    while n < 64 and (time.perf_counter() - t0) < args.cpu_budget:
        dense, emb, g = host[n % len(host)]
        p["tables"] = [emb[:, f, :] for f in range(model.F)]
        y, _, _ = O.deepfm(None, p, dt=np.float32, inputs=(dense, ids))
        if first is None:
            first = (np.asarray(y, np.float64), g)
        n += 1
    dt = time.perf_counter() - t0
    ref, g = first
    return {"value": n * B / dt, "unit": "samples/s", "cores": _cpu_threads(), "kind": "port",
            "sample": f"{n} batches x {B} samples of rank 0 (of {world}): numpy fp32 DeepFM forward (the reference "
                      f"TF graph restated; TF not installed) - EmbedLayer gather, FMLayer, DNNLayer "
                      f"429-256-128-64-1, sigmoid; the batch's rows copied from the shards (via rank 0's row "
                      f"exchange) into per-field host tables of the batch's own rows",
            "max_scaled_diff_vs_gpu": float(np.max(np.abs(g.reshape(ref.shape) - ref) / np.abs(ref)))}


def _world1_group():
    """A one-rank RCCL process group for the config-5 anchor inside the
    default N = 1 run (the driver's 1 -> N curve then has a same-workload
    point); MASTER_ADDR 127.0.0.1, a free port unless MASTER_PORT is set."""
    import socket
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(so.getsockname()[1])
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))


def _peer_leg_deepfm(args, world, model, dense_pool, ids_pool, out, step, rccl_dt):
    """Config 5's per-batch forward with both exchanges peer-mapped
    (ShardedDeepFM.use_peer_exchange: row ids through rs_peer_a2a, the
    owner's rows gathered straight into the requesters' mailboxes by
    rs_peer_gather_a2a — no rs_gather_rows launch, no row all-to-all).  The
    same 3 batches through RCCL and through the mailboxes must give
    bit-identical outputs on every rank; then the timed steps (graph-replayed).
    Failures are collective and reported; the RCCL value stands."""
    import torch.distributed as dist
    npool = ids_pool.shape[0]
    B = ids_pool.shape[1]
    try:
        ref = [model.forward((dense_pool[j], ids_pool[j]), check=True).clone() for j in range(3)]
        model.use_peer_exchange(spin_limit=BENCH_PEER_SPIN)
        got = [model.forward((dense_pool[j], ids_pool[j]), check=True) for j in range(3)]
        same = torch.tensor([int(all(torch.equal(a, b) for a, b in zip(ref, got)))], dtype=torch.int32,
                            device=ids_pool.device)
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        identical = bool(same.item())
        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        _barrier(world)
        dt, slot_ms = _timed_graph(step, args.steps, 0, world, chunk=16)
        fl = model.ops.bad_flag().clone()
        for ex in model.emb._peers.values():
            fl |= ex.err
        dist.all_reduce(fl, op=dist.ReduceOp.MAX)
        if int(fl.item()):
            raise RuntimeError(f"peer exchange: device error flag {int(fl.item()):#x}")
        res = {"samples_per_s": world * args.steps * B / dt, "ms_per_step": dt / args.steps * 1e3,
               "slot_ms": _max_over_ranks(slot_ms, world), "timing": "HIP graph replay (peer exchange captured)",
               "bit_identical_to_rccl": identical, "faster_and_identical": identical and dt < rccl_dt,
               "rccl_ms_per_step": rccl_dt / args.steps * 1e3,
               "protocol": "rs_shard_row_route, rs_peer_a2a of the row ids (one launch), rs_peer_gather_a2a (the "
                           "owner's rows straight into the requesters' mailboxes, one launch), rs_deepfm_fwd from "
                           "the mailbox"}
    except Exception as e:  # noqa: BLE001 — reported, the RCCL value stands
        res = {"error": repr(e)[:400]}
    finally:
        try:
            model.close_peer_exchange()
        except Exception as e:  # noqa: BLE001
            res = dict(res, close_error=repr(e)[:200])
    return res


def bench_sharded_deepfm(args, world, rank, lite=False):
    """BASELINE config 5 (nested as `config5` in the N > 1 line and as
    `config5_n1` at N = 1): DeepFM forward with ONE 1e8-row table (26 fields x 3,846,154 rows x 16 fp32 = 6.4 GB)
    row-sharded over the ranks, B = 4096 local samples per rank (weak
    scaling), DNN 429-256-128-64-1, FM k 10.  One step = ShardedDeepFM.forward
    on one batch: rs_shard_row_route -> RCCL all-to-all of row ids ->
    rs_gather_rows (owner) -> RCCL all-to-all of rows -> rs_deepfm_fwd from
    the exchange buffer (gather + FM + DNN tower + sigmoid, one launch).  The
    all-to-alls run at world 1 too (RCCL self-exchange).  Replayed from HIP
    graphs when RCCL capture works on every rank (collective decision)."""
    # config 5 is nested in every line (never its value): time at least
    # NESTED_MIN_STEPS batches whatever --steps is
    args = copy.copy(args)
    args.steps = max(args.steps, NESTED_MIN_STEPS)
    import torch.distributed as dist
    from recommender_system_amd.sharded import ShardedDeepFM
    B, F, k, nd, kfm = args.batch, 26, 16, 13, 10
    V = 3846154  # 26 x 3,846,154 = 1.0e8 rows
    vocabs = [V] * F
    dev = torch.device("cuda")
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    model = ShardedDeepFM(cols, kfm, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, device=dev, seed=SEED)
    model.emb._force_exchange = True
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + 101 + rank)
    npool = 16
    ids_pool = torch.randint(0, V, (npool, B, F), generator=g, device=dev, dtype=torch.int32)
    dense_pool = torch.rand(npool, B, nd, generator=g, device=dev)
    out = torch.empty(B, 1, device=dev)

    def step(i):
        j = i % npool
        model.forward((dense_pool[j], ids_pool[j]), check=False, out=out)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    _barrier(world)
    graphed, why = _graph_capturable(step, 0)
    if graphed:
        dt, slot_ms = _timed_graph(step, args.steps, 0, world, chunk=16)
        timing = "HIP graph replay (RCCL captured)"
    else:
        dt, _ = _timed(step, args.steps, 0, world, events=False)
        timing = f"eager launches ({why})"
    pipe = None
    if args.config5_pipelined:
        # pipelined stream (sharded.py pipe_step): batch t+1's route, id
        # all-to-all, owner gather and row all-to-all on a side stream while
        # batch t's fused kernel runs; two buffer slots, hub fork / join per
        # step.  Measured slower than the per-batch forward on one GPU
        # (DESIGN.md 4.6), so only on request.
        outs = [torch.empty(B, 1, device=dev) for _ in range(2)]

        def pstep(i):
            j, jn = i % npool, (i + 1) % npool
            model.pipe_step((dense_pool[j], outs[i % 2], i % 2), (ids_pool[jn], (i + 1) % 2))

        model.pipe_prologue(ids_pool[0], 0)
        for i in range(args.warmup):
            pstep(i)
        torch.cuda.synchronize()
        pgraphed, pwhy = _graph_capturable(pstep, 0, count=2)
        model.pipe_prologue(ids_pool[0], 0)
        if pgraphed:
            pdt, _ = _timed_graph(pstep, args.steps, 0, world, chunk=npool)
            ptiming = "HIP graph replay (RCCL captured, two streams)"
        else:
            pdt, _ = _timed(pstep, args.steps, 0, world, events=False)
            ptiming = f"eager launches ({pwhy})"
        pipe = {"protocol": "sharded.py pipe_step: batch t+1's exchange on a side stream beside batch t's "
                            "rs_deepfm_fwd (two buffer slots, fork / join on the step's stream)", "timing": ptiming,
                "samples_per_s": world * args.steps * B / pdt, "ms_per_step": pdt / args.steps * 1e3}
    f = model.ops.bad_flag()
    dist.all_reduce(f, op=dist.ReduceOp.MAX)
    if bool(f.item()):
        raise RuntimeError("sharded DeepFM bench: bad ids during timing")
    peer = _peer_leg_deepfm(args, world, model, dense_pool, ids_pool, out, step, dt) \
        if os.environ.get("RS_BENCH_PEER", "1") != "0" else {"skipped": "RS_BENCH_PEER=0"}
    # the fused DeepFM kernel alone, from the exchange buffer of the last step
    rb = model._rbufs(B)

    def finish(i):
        model.finish(dense_pool[i % npool], rb["got"], rb, out)

    fdt, fslot_ms = _timed_graph(finish, args.steps, 2, world, chunk=16)
    fin_ms = _max_over_ranks(fslot_ms, world)
    flops = B * 2 * (429 * 256 + 256 * 128 + 128 * 64 + 64)
    # value: the per-batch forward (the pipelined stream rides along when
    # asked for, never as the value)
    kind = "per_batch"
    ms = ums = dt / args.steps * 1e3
    S = model.emb.slot_stride
    roof = {"bound": "mfma", "achieved": flops / (fin_ms * 1e-3) / 1e12, "peak": PEAK_F32 / 1e12,
            "unit": "TFLOP/s", "frac": flops / (fin_ms * 1e-3) / PEAK_F32, "traffic": None,
            "kernel": "deepfm_ws (rs_deepfm_fwd_hm from the row-exchange buffer)",
            "kernel_ms": fin_ms, "dnn_flop_per_launch": flops,
            "kernel_ms_source": "HIP events around graph-replayed launches of the fused kernel alone"}
    exch = {"protocol": "field-range row records: rs_shard_row_route, RCCL all-to-all of row ids, "
                        "owner rs_gather_rows, RCCL all-to-all of rows, rs_deepfm_fwd with ids = slot_of",
            "timing": timing, "rows_per_rank": model.emb.rows_per_rank,
            "owner_field_ranges": model.emb.owner_field_ranges, "slots_per_sample_per_owner": S,
            "id_bytes_per_rank_each_way": world * B * S * 4,
            "row_bytes_per_rank_each_way": world * B * S * k * 4,
            "exchange_ms_per_step_unpipelined": ums - fin_ms}
    per_batch = {"samples_per_s": world * args.steps * B / dt, "ms_per_step": ums, "timing": timing,
                 "note": "ShardedDeepFM.forward per batch: route, all-to-all ids, gather, all-to-all rows, "
                         "rs_deepfm_fwd in sequence (the comparison for the pipelined value)"}
    cpu = _cpu_leg_config5(args, world, rank, model, dense_pool, ids_pool, out, B)
    res = {"samples_per_s": world * args.steps * B / dt, "ms_per_step": ms, "value_kind": kind,
           "per_batch": per_batch, "roofline": roof, "exchange": exch, "cpu_baseline": cpu, "peer_exchange": peer}
    if peer.get("faster_and_identical"):
        # the same forward with both exchanges peer-mapped (ids by rs_peer_a2a,
        # rows gathered into the requesters' mailboxes by rs_peer_gather_a2a):
        # bit-identical outputs, faster — the value; the RCCL per-batch numbers stay in per_batch
        res["samples_per_s"], res["ms_per_step"] = peer["samples_per_s"], peer["ms_per_step"]
        res["value_kind"] = "per_batch_peer_exchange"
    if pipe is not None:
        res["pipelined"] = pipe
    if lite:
        return res, V
    # secondary: the deduplicated exchange on Zipf(1.2) ids (hot rows repeat:
    # each owner receives every distinct row once per rank) and the training
    # step (forward exchange, local backward, reverse all-to-all of dL/drow,
    # owner row SGD, all-reduce of the replicated gradient)
    zrng = np.random.default_rng(SEED + 17 + rank)
    zipf_pool = torch.as_tensor(np.minimum(zrng.zipf(1.2, size=(npool, B, F)) - 1, V - 1).astype(np.int32),
                                device=dev)
    dmodel = ShardedDeepFM(cols, kfm, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, device=dev, seed=SEED,
                           dedup=0.5, table_init=False)
    dmodel.emb._force_exchange = True
    dmodel.emb.table_shard = model.emb.table_shard  # same shard (no second 1e8-row allocation)
    over = torch.zeros(1, dtype=torch.int32, device=dev)

    def step_zipf(m):
        def st(i):
            j = i % npool
            m.forward((dense_pool[j], zipf_pool[j]), check=False, out=out)
        return st

    nz = max(10, args.steps // 2)
    zfn, dfn = step_zipf(model), step_zipf(dmodel)
    for i in range(2):
        zfn(i)
        dfn(i)
    torch.cuda.synchronize()
    zg, zwhy = _graph_capturable(zfn, 0)
    dg, dwhy = _graph_capturable(dfn, 0)
    if zg and dg:  # both replayed from HIP graphs (collective decision)
        zdt, _ = _timed_graph(zfn, nz, 2, world, chunk=16)
        ddt, _ = _timed_graph(dfn, nz, 2, world, chunk=16)
        ztiming = "HIP graph replay (RCCL captured)"
    else:
        zdt, _ = _timed(zfn, nz, 2, world, events=False)
        ddt, _ = _timed(dfn, nz, 2, world, events=False)
        ztiming = f"eager launches ({zwhy or dwhy})"
    zedt, _ = _timed(zfn, nz, 2, world, events=False)
    dedt, _ = _timed(dfn, nz, 2, world, events=False)
    over += dmodel.ops.overflow_flag(dmodel._rbufs(B))
    dist.all_reduce(over, op=dist.ReduceOp.MAX)
    distinct = float(np.mean([sum(len(np.unique((model.emb.offsets[None, :].cpu().numpy() +
                                                 zipf_pool[j].cpu().numpy().astype(np.int64))[:, c]))
                                  for c in range(F)) for j in range(2)])) / (B * F)
    res["zipf_ids"] = {"distinct_lookup_fraction": distinct,
                       "field_range_records": {"samples_per_s": world * nz * B / zdt, "ms_per_step": zdt / nz * 1e3,
                                               "ms_per_step_eager": zedt / nz * 1e3,
                                               "row_bytes_per_rank_each_way": world * B * S * k * 4},
                       "dedup": {"samples_per_s": world * nz * B / ddt, "ms_per_step": ddt / nz * 1e3,
                                 "ms_per_step_eager": dedt / nz * 1e3,
                                 "capacity_fraction": 0.5, "overflow_seen": bool(over.item()),
                                 "row_bytes_per_rank_each_way": dmodel._rbufs(B)["n"] * k * 4},
                       "timing": ztiming,
                       "note": "Zipf(1.2) ids per field, clipped to the vocab; dedup = rs_shard_dedup_route (per-field "
                               "LDS hash, first-occurrence numbering, no sort): each owner receives each distinct "
                               "row once per rank"}
    if args.extras:
        labels = (torch.rand(npool, B, generator=g, device=dev) < 0.25).to(torch.float32)

        def train(i):
            j = i % npool
            model.train_step((dense_pool[j], ids_pool[j]), labels[j], lr=0.01, check=False)

        nt = max(10, args.steps // 4)
        tdt, _ = _timed(train, nt, 2, world, events=False)
        res["train_step"] = {"samples_per_s": world * nt * B / tdt, "ms_per_step": tdt / nt * 1e3,
                             "timing": "eager launches",
                             "note": "ShardedDeepFM.train_step: row exchange, local DeepFM backward (rs_gemm), "
                                     "rs_scatter_rows + reverse all-to-all of dL/drow, owner rs_embedding_sgd, "
                                     "all-reduce of the flat replicated gradient, SGD"}
    if world == 1:
        # what a world-1 job runs: no self-exchange, the fused DeepFM straight
        # from the (whole-table) shard
        model.emb._force_exchange = False
        ldt, lslot_ms = _timed_graph(step, args.steps, 2, world, chunk=16)
        model.emb._force_exchange = True
        res["world1_no_exchange"] = {
            "samples_per_s": args.steps * B / ldt, "ms_per_step": ldt / args.steps * 1e3, "slot_ms": lslot_ms,
            "timing": "HIP graph replay",
            "note": "world 1 without the RCCL self-exchange (ShardedDeepFM.forward -> rs_deepfm_fwd on the "
                    "shard); the exchange line above is the comparison"}
    return res, V


def _cpu_leg(args, rank, B, run_batch, n_pool, what, gpu_batch0=None, max_batches=64, kind_scale="scaled"):
    """`cpu_baseline` of a config line: the oracle's numpy fp32 op-for-op
    restatement of that config's step (the reference's TF graph; TF is not
    installed) on host copies of the same batches, a bounded sample of about
    --cpu-budget seconds on rank 0.  gpu_batch0(): the GPU step's output for
    batch 0, compared with the CPU's (max |a-b| / max(|b|, rms(b)))."""
    if not args.cpu_baseline or rank != 0:
        return None
    n, first, t0 = 0, None, time.perf_counter()
    while n < max_batches and (time.perf_counter() - t0) < args.cpu_budget:
        y = run_batch(n % n_pool)
        if first is None:
            first = np.asarray(y, np.float64)
        n += 1
    dt = time.perf_counter() - t0
    res = {"value": n * B / dt, "unit": "samples/s", "cores": _cpu_threads(), "kind": "port",
           "sample": f"{n} batches x {B} samples of this config's step ({what}); numpy fp32 oracle = the "
                     f"reference TF graph restated (TF not installed); host copies of the same tables and batches"}
    if gpu_batch0 is not None and first is not None:
        g = np.asarray(gpu_batch0(), np.float64).reshape(first.shape)
        rms = float(np.sqrt(np.mean(first ** 2))) or 1.0
        res["max_scaled_diff_vs_gpu"] = float(np.max(np.abs(g - first) / np.maximum(np.abs(first), rms)))
    return res


def _host_tables(embed_layer):
    t = embed_layer.table.detach().cpu().numpy()
    return [t[o:o + v] for o, v in zip(embed_layer.row_offsets, embed_layer.vocab_sizes)]


def _host_pool(ids_pool, dense_pool, n=8):
    return ids_pool[:n].cpu().numpy(), dense_pool[:n].cpu().numpy()


def _line(metric, value, unit, args, world, ms_per_step, config, roofline, extra=None, dtype="f32", hib=True):
    out = {"metric": metric, "value": value, "unit": unit, "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": hib, "scaling": "weak",
           "vs_baseline": None, "dtype": dtype, "data": "synthetic", "config": config, "roofline": roofline,
           "cpu_baseline": None}
    if extra:
        out.update(extra)
    return out


def _nested_args(args):
    """A config line nested in the N = 1 headline line (config3_n1 /
    config4_n1): at least NESTED_MIN_STEPS steps, a shorter CPU sample."""
    a = copy.copy(args)
    a.steps = max(args.steps, NESTED_MIN_STEPS)
    a.cpu_budget = min(args.cpu_budget, 5.0)
    return a


def bench_dcn(args, world, rank, nested=False):
    """Config 3: DCN CrossNet depth 3 on the DeepFM feature shape (26 x 1e6 x 16,
    13 dense, d = 429), B = 4096: step = rs_embed_cross_fwd (gather assembled in LDS + CrossNet, one
    launch); the two-launch path (rs_embed_gather + rs_cross_fwd) is reported beside it.
    nested: the config3_n1 leg of the N = 1 headline line (B 4096 whatever --batch)."""
    import recommender_system_amd as rs
    if nested:
        args = _nested_args(args)
        args.batch = 4096
    B, F, V, k, nd = args.batch, 26, int(args.vocab if args.vocab != 1e7 else 1e6), 16, 13
    dev = torch.device("cuda")
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    model = rs.DCN(cols, [256, 128, 64], 1, "relu", layer_num=3, embed_dim=k, seed=SEED, device=dev)
    ids_pool, dense_pool = _pool(B, [V] * F, nd, 64, dev)
    d = nd + F * k
    x = torch.empty(B, d, device=dev)
    y = torch.empty(B, d, device=dev)
    model.cross_layer.prepared(d)

    def gather(i):
        j = i % 64
        model.embed_layer.gather(ids_pool[j], dense=dense_pool[j], out=x, check_ids=False)

    def cross_only(i):
        model.cross_layer(x, out=y)

    def step(i):
        j = i % 64
        model.cross_fused((dense_pool[j], ids_pool[j]), out=y, check_ids=False)

    def two_launch(i):
        gather(i)
        cross_only(i)

    dt, slot = _timed_graph(step, args.steps, args.warmup, world)
    kern_ms = dt / args.steps * 1e3
    # algorithmic bytes of the fused launch: ids, dense, gathered rows, x_L out (+ weights)
    alg = B * (F * 4 + nd * 4 + F * k * 4 + d * 4) + 3 * 2 * d * 4
    ach = alg / (kern_ms * 1e-3)
    gather(0)
    _, cross_ms = _timed_graph(cross_only, args.steps, 5, world)
    dt_two, _ = _timed_graph(two_launch, args.steps, 5, world)
    useful = B * d * 3 * 2
    issued = ((B + 15) // 16) * ((d + 3) // 4) * 16 * 16 * 4 * 2
    n2 = max(NESTED_MIN_STEPS, args.steps // 5)

    def full(i):
        j = i % 64
        model((dense_pool[j], ids_pool[j]), check_ids=False)

    dt2, _ = _timed_graph(full, n2, args.warmup, world, chunk=16)
    cpu = None
    if args.cpu_baseline and rank == 0:
        from oracle import ctr_oracle as O
        tables = _host_tables(model.embed_layer)
        ws = [w.detach().cpu().numpy() for w in model.cross_layer.cross_weight]
        bs = [b.detach().cpu().numpy() for b in model.cross_layer.cross_bias]
        ids_h, dense_h = _host_pool(ids_pool, dense_pool)

        def cpu_step(j):
            x0 = np.concatenate([dense_h[j], O.embed_layer(ids_h[j], tables, np.float32)], 1)
            return O.cross_layer(x0, ws, bs, np.float32)

        def gpu0():
            step(0)
            return y.cpu().numpy()

        cpu = _cpu_leg(args, rank, B, cpu_step, 8, "EmbedLayer + concat + CrossLayer depth 3 -> x_L", gpu0)
    return _line("DCN CrossNet forward samples/sec @ batch 4096, 26 sparse x 1e6 vocab, dim 16, depth 3",
                 args.steps * B / dt, "samples/s", args, world, kern_ms,
                 {"workload": "dcn_embed+crossnet_depth3_fused", "global_batch": B, "d": d, "layer_num": 3,
                  "vocab_per_field": V, "parallelism": "dp1"},
                 {"bound": "hbm", "achieved": ach / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                  "frac": ach / PEAK_HBM, "traffic": _pmc_cfg("dcn"), "kernel": "embed_cross_ka", "kernel_ms": kern_ms,
                  "kernel_ms_source": "graph-replayed slot time per launch",
                  "algorithmic_bytes_per_launch": alg, "mfma_useful_flop_per_launch": useful,
                  "mfma_issued_flop_per_launch": issued, "mfma_useful_fraction_by_construction": useful / issued},
                 {"two_launch_gather_then_cross": {"samples_per_s": args.steps * B / dt_two,
                                                   "cross_mfma_kernel_ms": cross_ms,
                                                   "cross_mfma_hbm_frac": (B * 2 * d * 4) / (cross_ms * 1e-3) / PEAK_HBM},
                  "dcn_forward": {"samples_per_s": n2 * B / dt2, "ms_per_step": dt2 / n2 * 1e3},
                  "cpu_baseline": cpu})


def bench_din(args, world, rank, nested=False):
    """Config 4: DIN, Amazon-Electronics-shaped: B = 2048, T = 100, behaviour
    vocab 63,001, k = 8, 1 dense + user_id (192,404); step = behaviour-seq +
    candidate gathers + the attention-unit kernel.  nested: the config4_n1
    leg of the N = 1 headline line (no training step)."""
    import recommender_system_amd as rs
    if nested:
        args = _nested_args(args)
        args.batch = 4096
    B, T, k = 2048 if args.batch == 4096 else args.batch, 100, 8
    dev = torch.device("cuda")
    cols = [[{"feat": "age"}],
            [{"feat": "user_id", "feat_onehot_dim": 192404, "embed_dim": k},
             {"feat": "movies_seq", "feat_onehot_dim": 63001, "embed_dim": k}]]
    model = rs.DIN(cols, ["movies_seq"], seed=SEED, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(SEED)
    pool = []
    for _ in range(8):
        lens = torch.randint(1, T + 1, (B,), generator=g, device=dev)
        hist = torch.randint(1, 63001, (B, T), generator=g, device=dev)
        hist = torch.where(torch.arange(T, device=dev)[None, :] < lens[:, None], hist, torch.zeros_like(hist))
        pool.append({"age": torch.rand(B, 1, generator=g, device=dev),
                     "user_id": torch.randint(0, 192404, (B, 1), generator=g, device=dev),
                     "movie_id": torch.randint(1, 63001, (B, 1), generator=g, device=dev),
                     "movies_seq": hist})
    seq_layer = model.embed_seq_layers[0]
    att = model.att_layer
    seq = torch.empty(B * T, k, device=dev)
    item = torch.empty(B, k, device=dev)
    out = torch.empty(B, k, device=dev)
    masks = [(p["movies_seq"] != 0).to(torch.float32) for p in pool]
    model(pool[0], check_ids=False)  # builds the attention weights (alpha: [T, h])
    with torch.no_grad():
        for a in att.alphas:
            a.uniform_(-0.25, 0.25)

    table, V = seq_layer.table, 63001
    ws = torch.empty(B, T, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)

    def step(i):
        # the attention unit straight from ids: scores (MFMA) + masked softmax pool
        p = pool[i % 8]
        att.forward_ids(table, V, p["movies_seq"], p["movie_id"], err=err, out=out, scores=ws)

    def two_launch_materialised(i):
        p = pool[i % 8]
        seq_layer.gather(p["movies_seq"].reshape(B * T, 1), out=seq, check_ids=False)
        seq_layer.gather(p["movie_id"], out=item, check_ids=False)
        s3 = seq.view(B, T, k)
        att([item, s3, s3, masks[i % 8]], out=out)

    dt, _ = _timed_graph(step, args.steps, args.warmup, world)
    att_ms = dt / args.steps * 1e3
    dt_old, _ = _timed_graph(two_launch_materialised, args.steps, 5, world)
    flop = B * T * 2 * (4 * k * 80 + 80 * 40 + 40)  # reference formulation
    ach = flop / (att_ms * 1e-3)
    # issued MFMA flops: din_fused runs the MLP only on LIVE 16-position tiles
    # (>= 1 unmasked position; din.hip) - per position of a live tile the
    # regrouped layers issue 2 * (5*16*4*(k/4)*2 + 3*16*80) flops; with
    # U[1, T] lengths about half the positions are padding
    per_pos = 2 * (5 * 16 * 4 * (k // 4) * 2 + 3 * 16 * 80)
    live_pos = float(np.mean([float(((((m.sum(1) + 15) // 16) * 16).clamp(min=16)).sum()) for m in masks]))
    issued = live_pos * per_pos
    issued_all = B * ((T + 15) // 16) * 16 * per_pos
    # the same step on full-length histories (no padding: every tile live)
    full_pool = [dict(p, movies_seq=torch.randint(1, 63001, (B, T), generator=g, device=dev)) for p in pool[:2]]

    def step_full(i):
        p = full_pool[i % 2]
        att.forward_ids(table, V, p["movies_seq"], p["movie_id"], err=err, out=out, scores=ws)

    dtf_, _ = _timed_graph(step_full, args.steps, 5, world)
    full_ms = dtf_ / args.steps * 1e3
    n2 = max(NESTED_MIN_STEPS, args.steps // 5)

    def full(i):
        model(pool[i % 8], check_ids=False)

    dt2, _ = _timed_graph(full, n2, args.warmup, world, chunk=8)
    model.fused_call = False  # the two-launch DIN.call, for comparison
    dt2b, _ = _timed_graph(full, n2, args.warmup, world, chunk=8)
    model.fused_call = True
    cpu = None
    if args.cpu_baseline and rank == 0:
        from oracle import ctr_oracle as O
        table_h = table.detach().cpu().numpy()
        c_ = lambda t: t.detach().cpu().numpy()
        params = {"prelu": [(c_(att.kernels[i]), c_(att.biases[i]), c_(att.alphas[i])) for i in range(2)],
                  "out": (c_(att.out_kernel), c_(att.out_bias))}
        hist_h = [p["movies_seq"].cpu().numpy() for p in pool]
        cand_h = [p["movie_id"].cpu().numpy()[:, 0] for p in pool]

        def cpu_step(j):
            key = table_h[hist_h[j]]
            return O.attention(table_h[cand_h[j]], key, key, (hist_h[j] != 0).astype(np.float32), params, "prelu",
                               dt=np.float32)

        def gpu0():
            step(0)
            return out.cpu().numpy()

        cpu = _cpu_leg(args, rank, B, cpu_step, 8, "Attention 'prelu' (80, 40) on table[hist], table[cand], mask "
                                                  "= hist != 0", gpu0)
    # compile_fit's training step on DIN (DIN.train_step; after the forward
    # timings and the CPU leg: it moves the weights)
    labels = (torch.rand(8, B, generator=g, device=dev) < 0.25).to(torch.float32)

    def train(i):
        model.train_step(pool[i % 8], labels[i % 8], lr=0.01, check_ids=False)

    nt = max(10, args.steps // 10)
    tdt, ttiming = _train_timed(train, nt, world) if not nested else (None, None)
    return _line("DIN forward samples/sec @ batch 2048, behaviour seq len 100 (attention unit)",
                 args.steps * B / dt, "samples/s", args, world, att_ms,
                 {"workload": "din_attention_unit_from_ids", "global_batch": B, "seq_len": T, "embed_dim": k,
                  "att_hidden": [80, 40], "behaviour_vocab": 63001, "parallelism": "dp1"},
                 {"bound": "mfma", "achieved": ach / 1e12, "peak": PEAK_F32 / 1e12, "unit": "TFLOP/s",
                  "frac": ach / PEAK_F32, "traffic": _pmc_cfg("din"), "kernel": "din_fused", "kernel_ms": att_ms,
                  "kernel_ms_source": "graph-replayed step (one launch: scores, masked softmax, pool) / steps",
                  "useful_flop_per_launch": flop,
                  "useful_flop_note": "reference formulation B*T*2*(4k*80+80*40+40) over ALL T positions "
                                      "(SURVEY 8(d)); the kernel regroups layer 1 per sample (q(Wq+Wd) + "
                                      "key(Wk-Wd+diag(q)Wp)) and skips fully masked 16-position tiles, so it "
                                      "issues fewer",
                  "issued_mfma_flop_per_launch": issued,
                  "issued_note": "live tiles only: sum over samples of ceil(len/16)*16 positions (mean over the "
                                 "8-batch pool: %.0f of B*T = %d) x %d flops per position; check: PMC "
                                 "SQ_VALU_MFMA_BUSY_CYCLES x 64 (profiles/r6_pmc_din.json)" % (live_pos, B * T,
                                                                                               per_pos),
                  "issued_mfma_flop_if_every_tile_ran": issued_all,
                  "issued_mfma_tflops": issued / (att_ms * 1e-3) / 1e12,
                  "issued_frac_of_mfma_peak": issued / (att_ms * 1e-3) / PEAK_F32,
                  "no_padding": {"kernel_ms": full_ms, "frac": flop / (full_ms * 1e-3) / PEAK_F32,
                                 "issued_frac": issued_all / (full_ms * 1e-3) / PEAK_F32,
                                 "note": "every history full length (T valid positions, every tile live): the "
                                         "reference formulation's frac without padding"}},
                 {"materialised_keys_path": {"samples_per_s": args.steps * B / dt_old,
                                             "ms_per_step": dt_old / args.steps * 1e3},
                  "din_forward": {"samples_per_s": n2 * B / dt2, "ms_per_step": dt2 / n2 * 1e3,
                                  "two_launch_ms_per_step": dt2b / n2 * 1e3,
                                  "note": "graph-replayed full DIN.call (id checks off) as ONE launch "
                                          "(rs_din_forward_ids: the attention from ids, then BN + PReLU MLP + "
                                          "sigmoid head in the same workgroups, the other sparse rows and the "
                                          "dense features read into the tower tile); two_launch = the attention "
                                          "with the candidate rows (rs_din_attention_ids_cand_fwd), then the "
                                          "tower reading the pieces (rs_mlp_affine_pieces_fwd), bit-identical"},
                  "train_step": {"samples_per_s": nt * B / tdt, "ms_per_step": tdt / nt * 1e3,
                                 "timing": ttiming,
                                 "note": "DIN.train_step: gathers, attention Dense+PReLU layers over [B*T] rows, "
                                         "masked softmax pool, training-mode BN, PReLU DNN, full backward, SGD + "
                                         "row-sparse embedding SGD"} if not nested else None,
                  "cpu_baseline": cpu})


def bench_pnn(args, world, rank):
    """PNN inner-product path: fused gather + flatten + inner products, B=4096,
    26 x 1e6 x 16 -> [B, 416 + 325]."""
    import recommender_system_amd as rs
    B, F, V, k, nd = args.batch, 26, int(args.vocab if args.vocab != 1e7 else 1e6), 16, 13
    dev = torch.device("cuda")
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    model = rs.PNN(cols, "inner", [256, 128, 64], 1, embed_dim=k, seed=SEED, device=dev)
    ids_pool, dense_pool = _pool(B, [V] * F, nd, 64, dev)

    def step(i):
        model.product_inputs((dense_pool[i % 64], ids_pool[i % 64]), check_ids=False)

    dt, slot = _timed_graph(step, args.steps, args.warmup, world)
    alg = B * (F * 4 + F * k * 4 + (F * k + F * (F - 1) // 2) * 4)
    ach = alg / (slot * 1e-3)
    # mode 'both' (inner + OuterProductLayer, model/pnn.py:45-48) and the full PNN forward
    both = rs.PNN(cols, "both", [256, 128, 64], 1, embed_dim=k, seed=SEED, device=dev)
    P = F * (F - 1) // 2

    def step_both(i):
        both.product_inputs((dense_pool[i % 64], ids_pool[i % 64]), check_ids=False)

    def full(i):
        model((dense_pool[i % 64], ids_pool[i % 64]), check_ids=False)

    n2 = max(NESTED_MIN_STEPS, args.steps // 5)
    dtb, slotb = _timed_graph(step_both, n2, args.warmup, world)
    dtf, _ = _timed_graph(full, n2, args.warmup, world, chunk=16)
    cpu = None
    if args.cpu_baseline and rank == 0:
        from oracle import ctr_oracle as O
        tables = _host_tables(model.embed_layer)
        ids_h, dense_h = _host_pool(ids_pool, dense_pool)

        def cpu_step(j):
            flat = O.embed_layer(ids_h[j], tables, np.float32)
            return np.concatenate([flat, O.inner_product_layer(flat.reshape(B, F, k), np.float32)], 1)

        def gpu0():
            return model.product_inputs((dense_pool[0], ids_pool[0]), check_ids=False).cpu().numpy()

        cpu = _cpu_leg(args, rank, B, cpu_step, 8, "EmbedLayer (3-D) + InnerProductLayer -> [flat | inner]", gpu0)
    # the reference's PNN training loop (PNN.train_step, mode 'inner'; moves the weights)
    gl = torch.Generator(device=dev)
    gl.manual_seed(SEED + 5)
    labels = (torch.rand(16, B, generator=gl, device=dev) < 0.25).to(torch.float32)

    def train(i):
        model.train_step((dense_pool[i % 64], ids_pool[i % 64]), labels[i % 16], lr=0.01, check_ids=False)

    nt = max(10, args.steps // 10)
    tdt, ttiming = _train_timed(train, nt, world)
    return _line("PNN inner-product input samples/sec @ batch 4096, 26 sparse x 1e6 vocab, dim 16",
                 args.steps * B / dt, "samples/s", args, world, dt / args.steps * 1e3,
                 {"workload": "pnn_embed_inner_fused", "global_batch": B, "vocab_per_field": V, "parallelism": "dp1"},
                 {"bound": "hbm", "achieved": ach / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                  "frac": ach / PEAK_HBM, "traffic": _pmc_cfg("pnn"), "kernel": "inner_fast_ka", "kernel_ms": slot,
                  "algorithmic_bytes_per_launch": alg},
                 {"mode_both": {"samples_per_s": n2 * B / dtb, "kernel_ms": slotb,
                                "outer_mfma_tflops": B * P * k * k * 2 / (slotb * 1e-3) / 1e12,
                                "note": "[flat | inner | outer] in one launch (rs_embed_product_fwd)"},
                  "pnn_inner_forward": {"samples_per_s": n2 * B / dtf, "ms_per_step": dtf / n2 * 1e3,
                                        "note": "product inputs + DNN tower (rs_mlp_fwd, K = 741)"},
                  "train_step": {"samples_per_s": nt * B / tdt, "ms_per_step": tdt / nt * 1e3,
                                 "timing": ttiming,
                                 "note": "PNN.train_step (mode 'inner', model/pnn.py:74-81): [flat | inner], DNN "
                                         "fwd/bwd, Keras-broadcast BCE on the logit, inner-product backward, SGD + "
                                         "row-sparse embedding SGD"},
                  "cpu_baseline": cpu})


def _rank3_setup(args, k, nd=13):
    B, F = args.batch, 26
    V = int(args.vocab if args.vocab != 1e7 else 1e6)
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    ids_pool, dense_pool = _pool(B, [V] * F, nd, 64, torch.device("cuda"))
    return B, F, V, cols, ids_pool, dense_pool


_PMC_OF_WORKLOAD = {"nfm_embed_bi_interaction_fused": "nfm", "afm_att_fused": "afm", "ffm_fused": "ffm"}


def _hbm_line(metric, args, world, B, dt, slot, alg, workload, V, kernel, extra=None):
    ach = alg / (slot * 1e-3)
    cfg = _PMC_OF_WORKLOAD.get(workload)
    return _line(metric, args.steps * B / dt, "samples/s", args, world, dt / args.steps * 1e3,
                 {"workload": workload, "global_batch": B, "vocab_per_field": V, "parallelism": "dp1"},
                 {"bound": "hbm", "achieved": ach / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                  "frac": ach / PEAK_HBM, "traffic": _pmc_cfg(cfg) if cfg else None, "kernel": kernel,
                  "kernel_ms": slot, "algorithmic_bytes_per_launch": alg}, extra)


def bench_nfm(args, world, rank):
    """NFM (model/nfm.py, 3-D embeddings): ids -> rows -> bi-interaction ->
    [dense | pooled] in one launch (the headline), then BN + DNN tower."""
    import recommender_system_amd as rs
    k = 16
    B, F, V, cols, ids_pool, dense_pool = _rank3_setup(args, k)
    m = rs.NFM(cols, [256, 128, 64], 1, embed_dim=k, seed=SEED, device=torch.device("cuda"))

    def step(i):
        m.bi_interaction_input((dense_pool[i % 64], ids_pool[i % 64]), check_ids=False)

    def full(i):
        m((dense_pool[i % 64], ids_pool[i % 64]), check_ids=False)

    dt, slot = _timed_graph(step, args.steps, args.warmup, world)
    n2 = max(NESTED_MIN_STEPS, args.steps // 5)
    dtf, _ = _timed_graph(full, n2, args.warmup, world, chunk=16)
    alg = B * (F * 4 + F * k * 4 + 13 * 4 + (13 + k) * 4)
    cpu = None
    if args.cpu_baseline and rank == 0:
        from oracle import ctr_oracle as O
        tables = _host_tables(m.emb_layers)
        ids_h, dense_h = _host_pool(ids_pool, dense_pool)

        def cpu_step(j):
            flat = O.embed_layer(ids_h[j], tables, np.float32)
            return np.concatenate([dense_h[j], O.bi_interaction(flat.reshape(B, F, k), np.float32)], 1)

        def gpu0():
            return m.bi_interaction_input((dense_pool[0], ids_pool[0]), check_ids=False).cpu().numpy()

        cpu = _cpu_leg(args, rank, B, cpu_step, 8, "EmbedLayer (3-D) + Bi-Interaction -> [dense | pooled]", gpu0)
    return _hbm_line("NFM bi-interaction input samples/sec @ batch 4096, 26 sparse x 1e6 vocab, dim 16", args,
                     world, B, dt, slot, alg, "nfm_embed_bi_interaction_fused", V, "pair_pool_ksplit (sum)",
                     {"nfm_forward": {"samples_per_s": n2 * B / dtf, "ms_per_step": dtf / n2 * 1e3,
                                      "note": "bi-interaction launch + one tower launch (BN folded into the staging, DNN 29-256-128-64-1, Dense(1))"},
                      "cpu_baseline": cpu})


def bench_afm(args, world, rank):
    """AFM (model/afm.py): ids -> rows -> pair pooling -> Dense(1) -> 2 sigmoids
    in one launch; 'att' (== sum, the reference's size-1 softmax) and 'max'."""
    import recommender_system_amd as rs
    k = 16
    B, F, V, cols, ids_pool, dense_pool = _rank3_setup(args, k)
    dev = torch.device("cuda")
    m = rs.AFM(cols, "att", seed=SEED, device=dev)
    mx = rs.AFM(cols, "max", seed=SEED, device=dev)

    def step(i):
        m((dense_pool[i % 64], ids_pool[i % 64]), check_ids=False)

    def step_max(i):
        mx((dense_pool[i % 64], ids_pool[i % 64]), check_ids=False)

    dt, slot = _timed_graph(step, args.steps, args.warmup, world)
    dtm, slotm = _timed_graph(step_max, args.steps, args.warmup, world)
    alg = B * (F * 4 + F * k * 4 + 4)
    cpu = None
    if args.cpu_baseline and rank == 0:
        from oracle import ctr_oracle as O
        L = m.afm_layer
        c_ = lambda t: t.detach().cpu().numpy()
        m((dense_pool[0], ids_pool[0]), check_ids=False)  # attention weights are built on the first call
        a = L.attention_layer
        p = {"tables": _host_tables(L.embed_layer), "out_kernel": c_(L.output_layer.kernel),
             "out_bias": c_(L.output_layer.bias)}
        if a.attention_w is not None:
            p.update({"att_w_kernel": c_(a.attention_w.kernel), "att_w_bias": c_(a.attention_w.bias),
                      "att_h_kernel": c_(a.attention_h.kernel), "att_h_bias": c_(a.attention_h.bias)})
        ids_h, dense_h = _host_pool(ids_pool, dense_pool)

        def cpu_step(j):
            return O.afm(None, p, "att", dt=np.float32, inputs=(dense_h[j], ids_h[j]))[0]

        def gpu0():
            return m((dense_pool[0], ids_pool[0]), check_ids=False).cpu().numpy()

        cpu = _cpu_leg(args, rank, B, cpu_step, 8, "AFM.call 'att': Embedding per field, InteractionLayer [B, 325, "
                                                  "k], AttentionLayer, Dense(1), two sigmoids", gpu0)
    return _hbm_line("AFM forward samples/sec @ batch 4096, 26 sparse x 1e6 vocab, dim 16", args, world, B, dt,
                     slot, alg, "afm_att_fused", V, "pair_pool_ksplit (att == sum)",
                     {"mode_max": {"samples_per_s": args.steps * B / dtm, "kernel_ms": slotm,
                                   "note": "max over the 325 pair products per dim, in registers"},
                      "cpu_baseline": cpu})


def bench_ffm(args, world, rank):
    """FFM (model/ffm.py): one wave per sample gathers 26 rows of the
    [feature_num, 39, k] field-aware table (k = 8: 1,248-B rows)."""
    import recommender_system_amd as rs
    k = 8
    B, F, V, cols, ids_pool, dense_pool = _rank3_setup(args, k)
    m = rs.FFM(cols, k, seed=SEED, device=torch.device("cuda"))

    def step(i):
        m((dense_pool[i % 64], ids_pool[i % 64]))

    dt, slot = _timed_graph(step, args.steps, args.warmup, world)
    NF = 13 + F
    alg = B * (F * 4 + 13 * 4 + F * NF * k * 4 + F * 4 + 4)
    cpu = None
    if args.cpu_baseline and rank == 0:
        from oracle import ctr_oracle as O
        L = m.ffm
        ids_h, dense_h = _host_pool(ids_pool, dense_pool)
        # the touched rows of w / v only (the 32 GB field-aware table is not
        # copied to the host): per field, the rows of the pool's ids, ids remapped
        offs = np.concatenate([[0], np.cumsum(L.onehot_dims)[:-1]]).astype(np.int64)
        nd_ = L.nd
        cw, cv, rid, cdims = [L.w[:nd_].cpu().numpy()], [L.v[:nd_].cpu().numpy()], np.empty_like(ids_h), []
        for c in range(F):
            u, inv = np.unique(ids_h[:, :, c], return_inverse=True)
            rows = torch.as_tensor(nd_ + offs[c] + u, device=L.w.device)
            cw.append(L.w[rows].cpu().numpy())
            cv.append(L.v[rows].cpu().numpy())
            rid[:, :, c] = inv.reshape(ids_h.shape[:2])
            cdims.append(u.size)
        cw, cv, w0 = np.concatenate(cw), np.concatenate(cv), L.w0.cpu().numpy()

        def cpu_step(j):
            return O.sigmoid(O.ffm_layer_gather(dense_h[j], rid[j], cdims, w0, cw, cv, np.float32))

        def gpu0():
            return m((dense_pool[0], ids_pool[0])).cpu().numpy()

        cpu = _cpu_leg(args, rank, B, cpu_step, 8, "FFM.call: FFMLayer as row gathers of w / v (the one-hot x "
                                                  "never formed) + sigmoid; host copy holds the touched rows only",
                       gpu0)
    # compile_fit's step on FFM (FFM.train_step; after the forward timings and
    # the CPU leg: it moves the weights).  Keras' l2 on every row of v makes
    # the step a read + write of the whole table.
    gl = torch.Generator(device="cuda")
    gl.manual_seed(SEED + 9)
    labels = (torch.rand(16, B, generator=gl, device="cuda") < 0.25).to(torch.float32)

    def train(i):
        m.train_step((dense_pool[i % 64], ids_pool[i % 64]), labels[i % 16], lr=0.01)

    nt = max(5, args.steps // 20)
    tdt, ttiming = _train_timed(train, nt, world)
    vbytes = (13 + F * V) * NF * k * 4
    return _hbm_line("FFM forward samples/sec @ batch 4096, 26 sparse x 1e6 vocab, k 8", args, world, B, dt, slot,
                     alg, "ffm_fused", V, "ffm4_kernel",
                     {"table_GB": (13 + F * V) * NF * k * 4 / 1e9, "cpu_baseline": cpu,
                      "train_step": {"samples_per_s": nt * B / tdt, "ms_per_step": tdt / nt * 1e3,
                                     "l2_decay_hbm_frac": 2 * vbytes / (tdt / nt) / PEAK_HBM,
                                     "timing": ttiming,
                                     "note": "FFM.train_step: rs_ffm_train_fwd, dense-row rs_gemm, l2 decay of every "
                                             "row of w and v (2 x table bytes), row-sparse SGD of the looked-up rows"}})


def bench_io(args, world, rank):
    """Input path end to end: an RSCB file (page cache)
    -> pinned host buffers (native threaded copy) -> H2D on a copy stream ->
    the fused gather + FM kernel, overlapped by DeviceBatchLoader.  The value
    is the PCIe-inclusive rate (the headline's value keeps inputs resident)."""
    import tempfile

    import recommender_system_amd as rs
    from recommender_system_amd.batchio import DeviceBatchLoader, write_criteo
    B, F, V, k, nd = args.batch, 26, int(args.vocab), 16, 13
    dev = torch.device("cuda")
    nb = max(16, args.steps)
    rng = np.random.default_rng(SEED)
    N = nb * B
    dense = rng.random((N, nd), dtype=np.float32)
    ids = rng.integers(0, V, (N, F), dtype=np.int32)
    labels = rng.integers(0, 2, N).astype(np.float32)
    path = os.path.join(tempfile.gettempdir(), f"rs_bench_{os.getpid()}.rscb")
    write_criteo(path, dense, ids, labels, [V] * F)
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    model = rs.DeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=SEED, device=dev)
    loader = DeviceBatchLoader(path, B, dev, depth=3)
    try:
        for d, i, _ in loader:  # warm: page cache, pinned buffers, kernels
            model.fm_logit((d, i), check_ids=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for d, i, _ in loader:
            model.fm_logit((d, i), check_ids=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        # H2D alone (same slabs, no kernel) and the kernel alone (resident)
        t0 = time.perf_counter()
        for _ in loader:
            pass
        torch.cuda.synchronize()
        dt_io = time.perf_counter() - t0
        d0, i0 = torch.as_tensor(dense[:B], device=dev), torch.as_tensor(ids[:B], device=dev)
        for _ in range(20):
            model.fm_logit((d0, i0), check_ids=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(nb):
            model.fm_logit((d0, i0), check_ids=False)
        torch.cuda.synchronize()
        dt_k = time.perf_counter() - t0
    finally:
        os.unlink(path)
    h2d = B * (nd * 4 + F * 4 + 4)
    return _line("CTR forward samples/sec from an RSCB file (PCIe-inclusive), batch 4096, 26 sparse x 1e7 vocab, dim 16",
                 N / dt, "samples/s", args, world, dt / nb * 1e3,
                 {"workload": "rscb_file_to_fused_gather_fm", "global_batch": B, "vocab_per_field": V,
                  "batches": nb, "parallelism": "dp1"},
                 {"bound": "pcie", "achieved": h2d * nb / dt_io / 1e9, "peak": None, "unit": "GB/s", "frac": None,
                  "traffic": None, "kernel": "H2D of dense+ids+labels slabs", "h2d_bytes_per_batch": h2d},
                 {"io_only_samples_per_s": N / dt_io, "eager_kernel_only_samples_per_s": N / dt_k,
                  "note": "eager launches (host-side loader drives every batch); the headline value replays "
                          "graphs on resident inputs"})


def bench_fm_train(args, world, rank):
    """FM training step (compile_fit's SGD on FM):
    B = 4096 on 26 x 1e6 one-hot columns, k = 16 (config-2 shape), graph-
    replayed.  Keras' l2 regularisers give every row of w1 / v a gradient, so
    each step also rewrites the whole (n, 17) parameter block: that dense
    decay pass is the HBM-bound part; the sparse rows go through a sort +
    segmented sum.  Also timed: the reference's own scale (bundled-sample
    width 43,604, k = 8, batch 32)."""
    import recommender_system_amd as rs
    dev = torch.device("cuda")
    B, F, nd = args.batch, 26, 13
    V = int(args.vocab if args.vocab != 1e7 else 1e6)

    def setup(B, V, k, n_pool=16):
        vocab = np.full(F, V, np.int64)
        offs = np.concatenate([[0], np.cumsum(vocab)[:-1]])
        m = rs.FM(k, 1e-4, 1e-4, seed=SEED, device=dev)
        m.fm.build(nd + int(vocab.sum()))
        ids_pool, dense_pool = _pool(B, [V] * F, nd, n_pool, dev)
        labels = (torch.rand(n_pool, B, device=dev) < 0.25).to(torch.float32)
        o = torch.as_tensor(offs, device=dev)
        vo = torch.as_tensor(vocab, device=dev)

        def step(i):
            j = i % n_pool
            m.train_step(dense_pool[j], ids_pool[j], labels[j], o, vo, lr=0.01, check_ids=False)
        return m, step

    k = 16
    m, step = setup(B, V, k)
    dt, slot = _timed_graph(step, args.steps, args.warmup, world, chunk=16)
    # the same step on Zipf(1.05) ids: hot rows repeat thousands of times per
    # batch, so the sparse update's segment sums (one lane per column, fixed
    # order) carry long segments
    zrng = np.random.default_rng(SEED + 5)
    zpool = torch.as_tensor(np.minimum(zrng.zipf(1.05, size=(16, B, F)) - 1, V - 1).astype(np.int32), device=dev)
    zd = torch.rand(16, B, nd, device=dev)
    zl = (torch.rand(16, B, device=dev) < 0.25).to(torch.float32)
    zo = torch.as_tensor(np.arange(F, dtype=np.int64) * V, device=dev)
    zv = torch.full((F,), V, dtype=torch.int64, device=dev)

    def step_z(i):
        m.train_step(zd[i % 16], zpool[i % 16], zl[i % 16], zo, zv, lr=0.01, check_ids=False)

    dtz, _ = _timed_graph(step_z, args.steps, args.warmup, world, chunk=16)
    zmax = int(max(np.bincount(zpool[j, :, c].cpu().numpy()).max() for j in range(2) for c in range(F)))
    n_rows = nd + F * V
    decay = 2 * n_rows * (k + 1) * 4
    ach = decay / (slot * 1e-3)
    _, step_small = setup(32, 1677, 8)  # ~43,6xx one-hot columns, the bundled sample's width
    dts, slots = _timed_graph(step_small, args.steps, args.warmup, world, chunk=16)
    # DeepFM training step (config-2 model: 26 x 1e6 x 16 tables, DNN 256-128-64)
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": 16} for i in range(F)]]
    dfm = rs.DeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=16, seed=SEED, device=dev)
    ids_pool, dense_pool = _pool(B, [V] * F, nd, 16, dev)
    lab = (torch.rand(16, B, device=dev) < 0.25).to(torch.float32)

    def step_dfm(i):
        dfm.train_step((dense_pool[i % 16], ids_pool[i % 16]), lab[i % 16], lr=0.01, check_ids=False)

    n_d = max(10, args.steps // 5)
    dtd, _ = _timed_graph(step_dfm, n_d, args.warmup, world, chunk=16)
    del dfm
    # DCN training step (config-2 model: CrossNet 3 layers over d = 429, DNN 256-128-64 -> 1)
    dcn = rs.DCN(cols, [256, 128, 64], 1, "relu", 3, embed_dim=16, seed=SEED, device=dev)

    def step_dcn(i):
        dcn.train_step((dense_pool[i % 16], ids_pool[i % 16]), lab[i % 16], lr=0.01, check_ids=False)

    dtc, _ = _timed_graph(step_dcn, n_d, args.warmup, world, chunk=16)
    return _line("FM training samples/sec @ batch 4096, 26 x 1e6 one-hot columns, k 16 (SGD + l2, compile_fit)",
                 args.steps * B / dt, "samples/s", args, world, dt / args.steps * 1e3,
                 {"workload": "fm_train_step", "global_batch": B, "vocab_per_field": V, "k": k,
                  "parallelism": "dp1"},
                 {"bound": "hbm", "achieved": ach / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                  "frac": ach / PEAK_HBM, "traffic": None,
                  "kernel": "whole step; bytes = the l2 decay pass (read+write of w1 and v)", "kernel_ms": slot,
                  "decay_bytes_per_step": decay},
                 {"zipf_ids": {"samples_per_s": args.steps * B / dtz, "ms_per_step": dtz / args.steps * 1e3,
                               "max_lookups_of_one_row": zmax,
                               "note": "Zipf(1.05) ids per field (clipped to the vocab)"},
                  "deepfm_train": {"samples_per_s": n_d * B / dtd, "ms_per_step": dtd / n_d * 1e3,
                                   "note": "DeepFM.train_step: gather, DNN 429-256-128-64-1 fwd/bwd (rs_dense_fwd, "
                                           "rs_gemm), FM grads, SGD + l2, row-sparse embedding SGD"},
                  "dcn_train": {"samples_per_s": n_d * B / dtc, "ms_per_step": dtc / n_d * 1e3,
                                "note": "DCN.train_step: gather, CrossNet x3 fwd/bwd (rs_cross_train_fwd/_bwd), DNN "
                                        "429-256-128-64-1, output Dense, SGD + l2, row-sparse embedding SGD"},
                  "reference_scale": {"steps_per_s": args.steps / dts, "ms_per_step": dts / args.steps * 1e3,
                                      "note": "batch 32, 26 x 1,677 + 13 = 43,615 columns, k 8 (compile_fit's "
                                              "defaults on the bundled sample's width)"}})


def _train_timed(fn, n, world):
    """A single-GPU training step timed from HIP graphs of its launches when
    it captures (every launch is stream-ordered, no host sync inside), else
    eager; returns (seconds, timing label)."""
    try:
        dt, _ = _timed_graph(fn, n, 2, world, chunk=min(n, 8))
        return dt, "HIP graph replay"
    except Exception as e:  # noqa: BLE001 - a step that does not capture is timed eagerly
        torch.cuda.synchronize()
        dt, _ = _timed(fn, n, 2, world, events=False)
        return dt, f"eager launches ({type(e).__name__})"


def _pmc_cfg(cfg):
    """PMC HBM bytes per launch of a config line's dominant kernel
    (profiles/pmc_configs.json, scripts/gpu_pmc_configs.sh), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_configs.json")) as f:
            return json.load(f)[cfg]["hbm_bytes_per_launch"]
    except Exception:
        return None


def _pmc_traffic():
    p = os.path.join(ROOT, "profiles", "pmc_embed_fm.json")
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


_RESULT_OUT = None


def _emit(line):
    """The one JSON result line, on the process's original stdout (everything
    else — e.g. RCCL's version banner, which it prints to stdout at
    communicator init — goes to stderr, so stdout holds exactly that line)."""
    out = _RESULT_OUT if _RESULT_OUT is not None else sys.stdout
    out.write(json.dumps(line) + "\n")
    out.flush()


def main():
    global _RESULT_OUT
    import faulthandler
    faulthandler.enable()  # a native crash prints the Python stack
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--vocab", type=float, default=1e7)
    ap.add_argument("--config", default="hotpath")
    ap.add_argument("--cpu-baseline", dest="cpu_baseline", action="store_true", default=True)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--extras", action="store_true",
                    help="N > 1 / --sharded: also time the row-exchange protocol and the sharded training steps")
    ap.add_argument("--config5-pipelined", dest="config5_pipelined", action="store_true",
                    help="also time config 5's pipelined stream (slower than the per-batch forward on one GPU)")
    ap.add_argument("--no-config5", dest="no_config5", action="store_true",
                    help="skip the nested config-5 line (config5_n1 at N = 1, config5 at N > 1)")
    ap.add_argument("--no-configs34", dest="no_configs34", action="store_true",
                    help="skip the nested config-3 / config-4 lines of the N = 1 line")
    ap.add_argument("--sharded", action="store_true",
                    help="time the N > 1 line's row-sharded protocol even at world 1 (RCCL self-exchange)")
    args = ap.parse_args()
    _host_wait_mode(os.environ.get("RS_BENCH_SYNC", "spin"))
    world, rank = _dist_setup(args)
    if os.environ.get("RS_PEER_FENCES"):  # A/B of the peer exchange's ordering (rs_option RS_OPT_PEER_FENCES)
        from recommender_system_amd import _lib
        _lib.set_option(_lib.OPT_PEER_FENCES, int(os.environ["RS_PEER_FENCES"]))
    other = {"dcn": bench_dcn, "din": bench_din, "pnn": bench_pnn, "nfm": bench_nfm, "afm": bench_afm,
             "ffm": bench_ffm, "io": bench_io, "fm_train": bench_fm_train}
    if args.config in other:
        line = other[args.config](args, world, rank)
        if rank == 0:
            _emit(line)
        return
    if args.config == "deepfm1e6":
        args.vocab = 1e6
        args.no_config5 = True
    elif args.config != "hotpath":
        raise SystemExit(f"unknown --config {args.config}")
    dev_state = {"before": _device_state()}
    empty_slot = _empty_kernel_slot(world)
    res = bench_hotpath(args, world, rank)
    dev_state["after"] = _device_state()
    if rank == 0:
        line = {
            "metric": "CTR forward samples/sec @ batch 4096, 26 sparse×1e7 vocab, dim 16; %HBM roofline",
            "value": res["value"], "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": res["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "deepfm_embed_fm_hotpath", "global_batch": args.batch * world,
                       "batch_per_gpu": args.batch, "sparse_fields": 26, "vocab_per_field": int(args.vocab),
                       "embed_dim": 16, "fm_k": 10, "dense_features": 13, "ids": "int32 uniform per field"},
            "roofline": res["roofline"], "cpu_baseline": res["cpu_baseline"],
            "host_wait": os.environ.get("RS_BENCH_SYNC", "spin") if world == 1 else "default",
            "device_state": dev_state, "empty_kernel_slot_us": empty_slot,
        }
        if world == 1 and not args.sharded:
            line["config"].update({
                "parallelism": "dp1",
                "value_kind": "embed + FM logit (DeepFM's EmbedLayer + concat + FMLayer; no DNN, no sigmoid), one "
                              "unsharded rs_embed_fm_fwd launch per batch - the full DeepFM forward is "
                              "deepfm_forward, config 5 at N = 1 is config5_n1, the N > 1 protocol at world 1 is "
                              "fm_hotpath_sharded_n1"})
        else:
            line["config"].update({
                "parallelism": f"dp{world}+rowshard{world}",
                "table_rows_per_rank": res["rows_per_rank"],
                "value_kind": "embed + FM logit of the same workload with the 26 x 1e7 table row-sharded over the "
                              "ranks: per batch ONE exchange of [row ids | FM partials] records + ONE pipe launch "
                              "(combine | owner FM partials | field route); the exchange that produced the value: " +
                              res.get("exchange", "RCCL all_to_all") + " - the fastest of RCCL / peer-mapped, "
                              "one-deep (pipe_step: exchange then pipe) / two-deep (pipe2_step: exchange of t+1 "
                              "beside the pipe of t) whose logits are bit-identical to the one-deep RCCL step's, "
                              "all nested; config 5 (the DeepFM forward on the 1e8-row table) is nested as config5"})
        for key in ("concurrent_batches", "zipf_ids", "deepfm_forward", "config5_n1", "fm_hotpath_sharded_n1",
                    "config3_n1", "config4_n1", "streamed",
                    "config5", "protocol", "timing", "slot_ms", "unpipelined", "rows_protocol", "train_step",
                    "owner_field_ranges", "bytes_per_rank_each_way", "world1_no_exchange", "exchange",
                    "peer_exchange", "rccl_pipelined", "rccl_two_deep", "exchange_candidates_ms_per_step"):
            if key in res:
                line[key] = res[key]
        _emit(line)
    if _dist_on():
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
