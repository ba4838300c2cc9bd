#!/usr/bin/env python3
"""bench.py -- headline benchmark of the DWT -> percentile-threshold -> IDWT path on MI355X.

Workload (BASELINE.json configs[1]): bior3.3, level 5, 50th percentile
over the 20 Conv2d weights of ResNet-18 (11,166,912 fp32 weight coefficients per step;
synthetic kaiming-scaled values from csrc/wt_synth.h, generated on the device, resident in HBM
before the timed region).  One step = one wavelet_pruning-equivalent launch sequence over the
whole state_dict (every layer its own level/percentile, as dwt_pruning.py:130-174 does).
Multi-GPU (torchrun, one process per GPU): weak scaling, every rank prunes its own model
replica (independent objects, no data-path collective); the cfg4 variant (ONE model's layers
LPT-sharded + one RCCL all-gather) is measured as an extra leg and reported beside it.

Prints ONE JSON line on rank 0 (the driver contract).  --config cfg3/cfg5 run the other
single-GPU configs for DESIGN.md; they are not the headline line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "weight-coeffs/s for L5 bior3.3 DWT+thresh+IDWT; achieved HBM GB/s vs peak"
STAGES = ["forward_dwt", "k_window", "k_collect", "k_mask_select", "inverse_dwt"]
KERNEL_OF_STAGE = {"k_window": "k_window", "k_collect": "k_collect_t", "k_mask_select": "k_mask_select",
                   "forward_dwt": "k_fwd_level", "inverse_dwt": "k_inv_level"}
DWT_STAGES = ("forward_dwt", "inverse_dwt")  # one level launch per level: stage bytes = levels x per launch


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg3", "cfg5"])
    ap.add_argument("--blocks", type=int, default=8, help="cfg5: 4096^2 blocks per GPU")
    ap.add_argument("--graph-steps", type=int, default=10, help="steps captured per hipGraph replay")
    ap.add_argument("--stage-reps", type=int, default=30)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cold", action="store_true", help="also time with the Infinity Cache flushed")
    ap.add_argument("--flatten", action="store_true",
                    help="the 1-D flattened mode (WTP_FLATTEN; an extension, not the headline path)")
    ap.add_argument("--no-resident", action="store_true",
                    help="level-0 groups in the three-launch form instead of the one-launch k_resident")
    return ap.parse_args()


def workload(cfg, rank, blocks):
    from wavelettransforms_amd import workloads as W
    if cfg == "cfg2":
        ts = [(n, s, seed + 1000 * rank, tid, e) for (n, s, seed, tid, e) in W.resnet18_tensors(0)]
        return "resnet18_conv_state_dict", "bior3.3", 5, 50.0, ts
    if cfg == "cfg3":
        return "mnist_mlp_linear", "rbio2.2", 3, 50.0, W.mlp_tensors(3)
    ts = W.block_tensors(blocks * (rank + 1))[blocks * rank:]
    return "synthetic_4096x4096_blocks", "db8", 5, 50.0, ts


def stage_bytes(stage, n_w, pop, has_dwt):
    """Algorithmic bytes each stage must move (4 B read of w + 4 B write of w')."""
    if stage in ("forward_dwt", "inverse_dwt") and not has_dwt:
        return 0
    return {"forward_dwt": 4 * n_w + 4 * pop, "k_window": 0, "k_collect": 4 * pop,
            "k_mask_select": 8 * n_w if pop == n_w else 0, "inverse_dwt": 4 * pop + 4 * n_w}[stage]


def pmc_traffic(config, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summaries
    (profiles/pmc_<config>*.json, FETCH_SIZE x2 + WRITE_SIZE per DESIGN.md), if present."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_%s*.json" % config))):
        try:
            with open(path) as fh:
                d = json.load(fh)
            return d["kernels"][kernel]["hbm_bytes_per_launch"]
        except Exception:
            continue
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    from wavelettransforms_amd import _native as N
    from wavelettransforms_amd import engine

    if args.no_resident:
        engine.set_resident(False)
    name, wavelet, level, pct, ts = workload(args.config, rank, args.blocks)
    xs = [engine.synth(s, seed, tid, e, device=dev) for (_, s, seed, tid, e) in ts]
    outs = [torch.empty_like(x) for x in xs]
    n_w = sum(x.numel() for x in xs)

    def step():
        return engine.launch(xs, wavelet, level, pct, outs=outs, carry_level=False, flatten=args.flatten)

    for _ in range(max(1, args.warmup)):
        _, res = step()
    torch.cuda.synchronize()
    recs = engine.decode(res, len(xs))
    pop = sum(r["coeff_numel"] for r in recs)

    G = max(1, min(args.graph_steps, args.steps))
    graph = None
    if not args.no_graph:
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(G):
                step()
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()

    def timed(K, flush=None):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if graph is not None and flush is None:
            for _ in range(K // G):
                graph.replay()
            for _ in range(K % G):
                step()
        else:
            for _ in range(K):
                if flush is not None:
                    flush()
                step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([t], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
        return t

    K = args.steps
    T = timed(K)
    ms_per_step = T / K * 1e3
    value = world * n_w * K / T

    # ---- per-stage device durations: HIP events the library records between its launches on
    # the stream it runs on (wtp_set_stage_events); a spin kernel in front lets the whole call be
    # enqueued before it runs, so the events time the device, not the host; caches stay as warm
    # as in the timed loop (the same state rocprofv3's kernel trace of this command sees) ----
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(STAGES) + 1)]
    for e in evs:
        e.record()
    torch.cuda.synchronize()
    handles = (ctypes.c_void_p * len(evs))(*[e.cuda_event for e in evs])
    per = {st: [] for st in STAGES}
    N.lib().wtp_set_stage_events(handles, len(evs))
    try:
        for _ in range(args.stage_reps):
            torch.cuda._sleep(1_000_000)  # ~0.5 ms spin on the same stream
            step()
            torch.cuda.synchronize()
            for i, st in enumerate(STAGES):
                per[st].append(evs[i].elapsed_time(evs[i + 1]) * 1e3)  # us
    finally:
        N.lib().wtp_set_stage_events(None, 0)
    stage_us = {st: float(np.median(v)) for st, v in per.items()}
    # level-0 groups within the co-resident grid run as ONE launch (k_resident): the library
    # records stages 1-3 back to back in front of it, so "k_mask_select" times that launch
    resident = (not args.no_resident and all(r["eff_level"] == 0 for r in recs) and len(xs) <= 24
                and sum(-(-x.numel() // 49152) for x in xs) <= engine.resident_capacity())
    kernel_of = dict(KERNEL_OF_STAGE, k_mask_select="k_resident") if resident else KERNEL_OF_STAGE
    if resident:
        stage_us = {("k_resident" if st == "k_mask_select" else st): v for st, v in stage_us.items()
                    if st not in ("k_window", "k_collect")}
    has_dwt = any(r["eff_level"] > 0 for r in recs)

    def per_stage(st):
        return float(np.median(per[st]))
    dom = max((st for st in STAGES if stage_bytes(st, n_w, pop, has_dwt) > 0), key=lambda st: per_stage(st))
    dom_bytes = stage_bytes(dom, n_w, pop, has_dwt)
    achieved = dom_bytes / (per_stage(dom) * 1e-6) / 1e9
    # a DWT stage is one launch per level (every level of these workloads takes the tiled path in
    # one grouped launch); the PMC summary holds bytes per launch averaged over the levels
    dom_launches = max(r["eff_level"] for r in recs) if dom in DWT_STAGES else 1
    dom_traffic = pmc_traffic(args.config, kernel_of.get(dom, dom))

    cold = None
    if args.cold:
        flush_buf = torch.empty(512 << 20 >> 2, dtype=torch.float32, device=dev)
        Kc = max(10, K // 10)
        # time flush alone, subtract it (the flush is not part of the path)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(Kc):
            flush_buf.fill_(1.0)
        torch.cuda.synchronize()
        tf = time.perf_counter() - t0
        tc = timed(Kc, flush=lambda: flush_buf.fill_(1.0))
        cold = {"ms_per_step": (tc - tf) / Kc * 1e3, "note": "Infinity Cache flushed by a 512 MiB write per step"}

    # ---- cfg4: one model LPT-sharded over the ranks + one RCCL all-gather ----
    sharded = None
    if world > 1 and args.config == "cfg2":
        from wavelettransforms_amd.sharding import prune_sharded
        base = [engine.synth(s, seed, tid, e, device=dev) for (_, s, seed, tid, e) in workload("cfg2", 0, 0)[4]]

        def fn(sub):
            return engine.prune(sub, wavelet, level, pct, carry_level=False)

        for _ in range(3):
            prune_sharded(base, wavelet, level, pct, fn)
        dist.barrier()
        torch.cuda.synchronize()
        Ks = 20
        t0 = time.perf_counter()
        for _ in range(Ks):
            _, _, plan = prune_sharded(base, wavelet, level, pct, fn)
        torch.cuda.synchronize()
        dist.barrier()
        ts_ = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(ts_, op=dist.ReduceOp.MAX)
        sharded = {"ms_per_step": float(ts_.item()) / Ks * 1e3, "max_rank_weights": int(plan.max_shard),
                   "note": "one model, LPT layer shards + all_gather_into_tensor (RCCL), host-synchronous"}

    # ---- CPU baseline: the C oracle (port of the reference's arithmetic) on host cores ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import oracle as O
        host = [O.synth(s, seed, tid, e) for (_, s, seed, tid, e) in ts]
        O.prune_batch(host[:1], wavelet, level, pct)
        reps, t0 = 0, time.perf_counter()
        while True:
            O.prune_batch(host, wavelet, level, pct, nthreads=1)
            reps += 1
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        tcpu = time.perf_counter() - t0
        cpu = {"value": n_w * reps / tcpu, "unit": "weight-coeffs/s", "cores": 1, "kind": "port",
               "sample": "%d full passes over the %s workload (%d weights) with the single-threaded C "
                         "restatement (oracle/wtprune_oracle.c), %.1f s" % (reps, name, n_w, tcpu)}

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "weight-coeffs/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (splitmix64 Irwin-Hall, kaiming-scaled)",
            "config": {"workload": name, "config": args.config, "wavelet": wavelet, "level": level,
                       "percentile": pct, "weights_per_gpu_step": n_w, "coeffs_per_gpu_step": pop,
                       "tensors": len(xs), "eff_levels": sorted({r["eff_level"] for r in recs}),
                       "graph_steps": G if graph is not None else 0, "parallelism": "replica%d" % world,
                       "transform": "1-D flattened (extension)" if args.flatten else "2-D over (kh, kw) (reference)"},
            "pipeline_hbm_gbs": 8 * n_w * K / T / 1e9,
            "roofline": {"bound": "hbm", "kernel": kernel_of.get(dom, dom), "stage": dom,
                         "launches_per_stage": dom_launches, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": (None if dom_traffic is None else dom_traffic * dom_launches),
                         "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_us": per_stage(dom)},
            "stage_us": stage_us,
            "cpu_baseline": cpu,
        }
        if cold:
            line["cold_mall"] = cold
        if sharded:
            line["cfg4_sharded_one_model"] = sharded
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
