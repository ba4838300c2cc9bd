#!/usr/bin/env python3
"""bench.py -- headline benchmark of the DWT -> percentile-threshold -> IDWT path on MI355X.

Workload (BASELINE.json configs[1]): bior3.3, level 5, 50th percentile over
the 20 Conv2d weights of ResNet-18 (11,166,912 fp32 weight coefficients per model; synthetic
kaiming-scaled values from csrc/wt_synth.h, generated on the device, resident in HBM before the
timed region).  One step = one wavelet_pruning-equivalent pass over the whole state_dict (every
layer its own level and percentile, dwt_pruning.py:130-174).

--gpus N (N > 1): unless WORLD_SIZE is set (torchrun), N rank processes are started here, before
anything touches the GPU (python -m torch.distributed.run on 127.0.0.1), one per GPU.  The
headline at N > 1 is north_star's split, BASELINE configs[3] (cfg4): ONE model's layers
LPT-sharded over the ranks, each rank pruning its layers straight into its region of the flat
state_dict buffer, then ONE full-mesh exchange of the unpadded regions (an RCCL group of
point-to-point copies over xGMI) that reassembles the pruned state_dict on every rank -- strong
scaling of one model (end-to-end per step = compute + all-gather, max over ranks).  The replica
leg (every rank prunes its own model, no collective: weak scaling) is reported beside it.
--config cfg5 (BASELINE configs[4]): 64 blocks of 4096^2 (db8 level 5) split over the ranks
(strong scaling); --config cfg3 the MLP (launch-latency regime).

Prints ONE JSON line on rank 0 (the driver contract).
"""
import argparse
import ctypes
import glob
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.0  # one xGMI peer link, per direction (MI355X: 7 links per GPU)
# FP32 vector rate without FMA contraction, mul + add counted as two flops: MEASURED on MI355X with
# independent v_pk_mul_f32 / v_pk_add_f32 chains at >= 2 waves per SIMD (tools/mb/pkrate.hip,
# profiles/r03_valu_nofma_rate.txt: 128 TF/s packed, 120 TF/s scalar); SURVEY.md 8(d)'s 78.6 was
# an estimate (half the FMA spec)
VALU_NOFMA_TFLOPS = 128.0
METRIC = "weight-coeffs/s for L5 bior3.3 DWT+thresh+IDWT; achieved HBM GB/s vs peak"
STAGES = ["forward_dwt", "k_window", "k_collect", "k_mask_select", "inverse_dwt"]
KERNEL_OF_STAGE = {"k_window": "k_window", "k_collect": "k_collect_t", "k_mask_select": "k_mask_select",
                   "forward_dwt": "k_fwd_int+k_fwd_level", "inverse_dwt": "k_inv_int+k_inv_level"}
DWT_STAGES = ("forward_dwt", "inverse_dwt")
CFG5_BLOCKS = 64
DB8_L5_FLOP_PER_ELEM = 170.5  # 4 F sum_k 4^-k MACs, no FMA, F = 16, L = 5


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg3", "cfg5"])
    ap.add_argument("--blocks", type=int, default=CFG5_BLOCKS, help="cfg5: 4096^2 blocks in all (split over ranks)")
    ap.add_argument("--graph-steps", type=int, default=10, help="steps captured per hipGraph replay")
    ap.add_argument("--replays", type=int, default=60, help="graph replays timed one by one (p10/p50/p90)")
    ap.add_argument("--stamp-reps", type=int, default=50, help="launches timed by in-kernel stamps")
    ap.add_argument("--stage-reps", type=int, default=20,
                    help="calls timed stage by stage (0: no stage leg and no roofline object; tools/pmc_run.sh)")
    ap.add_argument("--cold-reps", type=int, default=30)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cold", action="store_true")
    ap.add_argument("--flatten", action="store_true",
                    help="the 1-D flattened mode (WTP_FLATTEN; an extension, not the headline path)")
    ap.add_argument("--no-resident", action="store_true",
                    help="level-0 groups in the three-launch form instead of the one-launch k_resident")
    ap.add_argument("--no-interior", action="store_true",
                    help="run every filter-bank tile in the general kernel (wtp_set_interior(0); A/B only)")
    ap.add_argument("--frame-general", action="store_true",
                    help="run the frame of edge tiles in the general kernel (wtp_set_interior(1); A/B only)")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="wtp_set_pipeline mode for multi-group calls (default: the library's; A/B only)")
    ap.add_argument("--no-fused-select", action="store_true",
                    help="cfg5-sized groups: the window / collect / select passes over the packed array instead of "
                         "the fused selection (wtp_set_fused_select(0); A/B only)")
    ap.add_argument("--frame-apart", action="store_true",
                    help="the frame of edge tiles in a launch of its own (wtp_set_interior(2); A/B only)")
    ap.add_argument("--no-rocprof", action="store_true", help="skip the in-run rocprofv3 kernel-stats child")
    ap.add_argument("--exchange", default="p2p", choices=["p2p", "allgather"],
                    help="N > 1 cfg4 reassembly: full-mesh point-to-point copies of the unpadded regions (default) "
                         "or one in-place all_gather_into_tensor of the padded regions")
    ap.add_argument("--profile-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """Start n rank processes (one per GPU) and relay their exit status.  Runs before this process
    touches the GPU: the ranks are children, nothing is exec'ed over a GPU-initialised process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def pmc_traffic(config, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this config's
    current kernels (profiles/pmc_<config>.json: 2 x FETCH_SIZE + WRITE_SIZE, separate passes)."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % config)
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d["kernels"][kernel]["hbm_bytes_per_launch"], os.path.relpath(path, ROOT), d.get("source")
    except Exception:
        return None, None, None


def rocprof_child(args, timeout=240):
    """The headline step loop of this very configuration under rocprofv3 --kernel-trace --stats,
    run as a child process BEFORE this process touches the GPU; returns {kernel name: (calls,
    average ns)} from its kernel-stats summary, or None if the profiler is unavailable."""
    import csv
    import shutil
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    d = tempfile.mkdtemp(prefix="wtp_bench_prof_", dir="/tmp")
    cmd = [prof, "--kernel-trace", "--stats", "-d", d, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.abspath(__file__), "--profile-child", "--config", args.config,
           "--steps", str(max(args.steps, 200)), "--warmup", str(args.warmup), "--blocks", str(args.blocks),
           "--graph-steps", str(args.graph_steps)]
    if args.no_graph:
        cmd.append("--no-graph")
    if args.flatten:
        cmd.append("--flatten")
    if args.no_resident:
        cmd.append("--no-resident")
    if args.no_interior:
        cmd.append("--no-interior")
    if args.frame_general:
        cmd.append("--frame-general")
    if args.frame_apart:
        cmd.append("--frame-apart")
    if args.pipeline is not None:
        cmd += ["--pipeline", str(args.pipeline)]
    if args.no_fused_select:
        cmd.append("--no-fused-select")
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                       timeout=timeout, check=True)
        stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        keep = os.environ.get("WTP_BENCH_TRACE_DIR")  # lab: keep the child's trace and stats
        if keep:
            os.makedirs(keep, exist_ok=True)
            for f in glob.glob(os.path.join(d, "**", "*kernel_*.csv"), recursive=True):
                shutil.copy(f, os.path.join(keep, os.path.basename(f)))
        out = {}
        with open(stats[0]) as fh:
            for row in csv.DictReader(fh):
                out[row["Name"]] = (int(row["Calls"]), float(row["TotalDurationNs"]))
        return out
    except Exception:
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


def rocprof_kernel(stats, kernel):
    """(total ns, launches) of the wtp kernel named `kernel` (every template instance) in a
    rocprof_child summary; (0.0, 0) if absent."""
    calls, total = 0, 0.0
    want = {"wtp::" + k for k in kernel.split("+")}  # a stage's kernels ("a+b": interior + frame)
    for name, (c, t) in (stats or {}).items():
        base = name.split("(")[0].split("<")[0].replace("void ", "").strip()
        if base in want:
            calls += c
            total += t
    return total, calls


def child_steps(args):
    """Steps the rocprof child executes: warmup, the side-stream step and two warm replays of the
    graph (when one is captured), then the timed steps."""
    K = max(args.steps, 200)
    G = max(1, min(args.graph_steps, K))
    return args.warmup + K + (0 if args.no_graph else 1 + 2 * G)


def dwt_stage_work(shapes_levels, F):
    """Per step, over the tensors' (shape, effective level) pairs: the bytes each tiled filter-bank
    stage moves at its minimum -- forward level k reads its R_{k-1} x C_{k-1} input and writes four
    R_k x C_k subbands; inverse level k reads four subbands and writes its 2R_k x 2C_k output (the
    last one cropped to H x W) -- and the flops (no FMA) each stage computes: 8 F R_k C_k MACs per
    level and batch item, forward and inverse alike (pywt periodization: N_k = ceil(N_{k-1} / 2))."""
    fwd = inv = flops = 0
    for shape, L in shapes_levels:
        if L <= 0 or len(shape) < 2:
            continue
        H, W = int(shape[-2]), int(shape[-1])
        B = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
        R, C = [H], [W]
        for _ in range(L):
            R.append((R[-1] + 1) // 2)
            C.append((C[-1] + 1) // 2)
        for k in range(1, L + 1):
            fwd += 4 * B * (R[k - 1] * C[k - 1] + 4 * R[k] * C[k])
            inv += 4 * B * (4 * R[k] * C[k] + (H * W if k == 1 else 4 * R[k] * C[k]))
            flops += 2 * 8 * F * R[k] * C[k] * B  # per stage
    return {"forward_dwt": fwd, "inverse_dwt": inv, "flops_per_stage": flops}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        n = min(n, int(omp))  # the box's CPU share (16 per GPU there)
    return max(1, n)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    # single process: first the kernel-stats child (rocprofv3 over this same step loop), before
    # this process touches the GPU; its per-kernel average is the roofline's launch duration
    prof_stats = None
    if (not args.profile_child and not args.no_rocprof and int(os.environ.get("WORLD_SIZE", "1")) == 1):
        prof_stats = rocprof_child(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # WTP_BENCH_REHEARSAL=1: the N > 1 code path on a one-GPU box (every rank on device 0, gloo
    # instead of RCCL) -- a functional rehearsal only, its numbers mean nothing
    rehearsal = os.environ.get("WTP_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from wavelettransforms_amd import _native as N
    from wavelettransforms_amd import engine
    from wavelettransforms_amd import workloads as W
    from wavelettransforms_amd.sharding import REC_BYTES, ShardPlan, _Shard, assemble, exchange

    L = N.lib()
    if args.no_resident:
        engine.set_resident(False)
    if args.no_interior:
        engine.set_interior(False)
    elif args.frame_general:
        engine.set_interior(1)
    elif args.frame_apart:
        engine.set_interior(2)
    if args.pipeline is not None:
        engine.set_pipeline(args.pipeline)
    if args.no_fused_select:
        engine.set_fused_select(False)

    # ---------------------------------------------------------------- workload
    if args.config == "cfg2":
        name, wavelet, level, pct = "resnet18_conv_state_dict", "bior3.3", 5, 50.0
        model = [(s, seed, tid, e) for (_, s, seed, tid, e) in W.resnet18_tensors(0)]
    elif args.config == "cfg3":
        name, wavelet, level, pct = "mnist_mlp_linear", "rbio2.2", 3, 50.0
        model = [(s, seed, tid, e) for (_, s, seed, tid, e) in W.mlp_tensors(3)]
    else:
        name, wavelet, level, pct = "synthetic_4096x4096_blocks", "db8", 5, 50.0
        nb = max(world, args.blocks)
        per = nb // world
        model = [(s, seed, tid, e) for (_, s, seed, tid, e) in W.block_tensors(per * world)]
    sharded = world > 1 and args.config in ("cfg2", "cfg3")   # cfg4: one model over the ranks
    if args.config == "cfg5":
        mine = model[rank * per:(rank + 1) * per]               # cfg5: the blocks split over the ranks
    elif sharded:
        plan = ShardPlan([s for (s, *_) in model], world, args.exchange)
        mine = [model[i] for i in plan.mine[rank]]
    else:
        mine = model
    xs_all = [engine.synth(s, seed, tid, e, device=dev) for (s, seed, tid, e) in
              (model if sharded else mine)]
    n_model = sum(int(np.prod(s)) for (s, *_) in model)          # weights of the whole job per step
    n_w = sum(x.numel() for x in (xs_all if not sharded else [xs_all[i] for i in plan.mine[rank]]))

    if sharded:
        shard = _Shard(xs_all, plan, rank, dev)  # its region of the flat state_dict buffer shard.full

        def compute():
            if shard.mine:
                shard.run(shard.mine, wavelet, level, pct)

        def gather():
            exchange(shard.full, plan, rank)

        def step():
            compute()
            gather()
        xs = [xs_all[i] for i in plan.mine[rank]]
    else:
        xs = xs_all
        outs = [torch.empty_like(x) for x in xs]
        res_buf = torch.empty(max(1, len(xs)) * REC_BYTES, dtype=torch.uint8, device=dev)

        def step():
            engine.launch(xs, wavelet, level, pct, outs=outs, carry_level=False, flatten=args.flatten,
                          results=res_buf)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    if sharded:
        _, recs_all = assemble(shard.full, plan)
        recs = [recs_all[i] for i in plan.mine[rank]]
    else:
        host = res_buf.cpu().numpy().view(engine.RESULT_DTYPE)[:len(xs)]
        recs = [{k: r[k].item() for k in engine.RESULT_DTYPE.names} for r in host]
    faults = sum(1 for r in recs if r["path"] == engine.MODE_FAULT)
    pop = sum(r["coeff_numel"] for r in recs)
    resident = (not args.no_resident and not args.flatten and recs and all(r["eff_level"] == 0 for r in recs)
                and len(xs) <= 24 and sum(-(-x.numel() // 49152) for x in xs) <= engine.resident_capacity())
    has_dwt = any(r["eff_level"] > 0 for r in recs)
    # the whole call as one k_small launch (csrc/small.hip): small 2-D calls, e.g. cfg3
    small = bool(recs) and not sharded and all(r["path"] == engine.MODE_SMALL for r in recs)

    # WTP_CRASH_DIAG=<dir>: Python-level fault handler into <dir>/faulthandler.txt and a snapshot
    # of this process's memory map in <dir>/maps.txt taken just before the graph is captured, so
    # the native frames of a crash inside a graph replay can be mapped to their libraries
    diag = os.environ.get("WTP_CRASH_DIAG")
    if diag:
        import faulthandler
        os.makedirs(diag, exist_ok=True)
        _fh = open(os.path.join(diag, "faulthandler.txt"), "w")
        faulthandler.enable(file=_fh, all_threads=True)

    # ------------------------------------------------- hipGraph (single-process configs)
    G = max(1, min(args.graph_steps, args.steps))
    graph = None
    if not args.no_graph and world == 1:
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        # captured on the warmed stream: its workspace (engine.workspace, per stream) exists, so no
        # zero-fill of a fresh workspace is captured into the graph (round 4's lines replayed one
        # per replay: cfg5 a ~17 GB memset, 0.34 ms per step; cfg2 6 us per 10 steps)
        with torch.cuda.graph(graph, stream=s):
            for _ in range(G):
                step()
        if diag:
            with open("/proc/self/maps") as fi, open(os.path.join(diag, "maps.txt"), "w") as fo:
                fo.write(fi.read())
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()

    def max_over_ranks(t):
        if world == 1:
            return t
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    def timed(K, fn=None):
        fn = fn or step
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if graph is not None and fn is step:
            for _ in range(K // G):
                graph.replay()
            for _ in range(K % G):
                step()
        else:
            for _ in range(K):
                fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return max_over_ranks(time.perf_counter() - t0)

    def faulted_now():
        """Records of the last step that read MODE_FAULT (a resident wait timed out: nothing was
        stored for that tensor and the step absorbed the bound) -- the line is marked, not trusted."""
        if sharded:
            _, rr = assemble(shard.full, plan)
            return sum(1 for r in rr if r["path"] == engine.MODE_FAULT)
        return int(engine.fault_mask(res_buf, len(xs)).sum()) if xs else 0

    # ------------------------------------------------------------ the headline
    K = args.steps
    T = timed(K)  # exactly K steps between barrier + synchronize, max over ranks
    ms_per_step = T / K * 1e3
    value = n_model * K / T
    timed_region = {"steps": K, "ms_per_step": ms_per_step, "value": value}
    if args.profile_child:
        return
    faults_timed = faulted_now()

    # per-replay distribution (>= 50 replays of G steps, each bracketed by events on the stream);
    # with a graph the headline value and ms_per_step are its p50, so that a short --steps (the
    # driver's 20 = 2 replays) cannot hinge on one or two replays
    dist_ms = None
    value_src = "the K-step timed region (barrier + synchronize on both sides, max over ranks)"
    if graph is not None:
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(max(50, args.replays))]
        for a, b in evs:
            a.record()
            graph.replay()
            b.record()
        torch.cuda.synchronize()
        per = np.array([a.elapsed_time(b) / G for a, b in evs])
        dist_ms = {"replays": len(evs), "steps_per_replay": G, "p10": float(np.percentile(per, 10)),
                   "p50": float(np.percentile(per, 50)), "p90": float(np.percentile(per, 90))}
        ms_per_step = dist_ms["p50"]
        value = n_model / (ms_per_step * 1e-3)
        value_src = ("p50 of %d graph replays of %d steps each, HIP events on the replay stream; the K-step timed "
                     "region is reported beside it as timed_region" % (len(evs), G))
    faults_timed += faulted_now()

    # ------------------------------------- dominant kernel: in-kernel launch span
    def stamp_spans(reps, before=None):
        st = torch.empty((reps, 2), dtype=torch.int64, device=dev)
        st[:, 0] = -1  # ~0 as unsigned
        st[:, 1] = 0
        torch.cuda.synchronize()
        base = st.data_ptr()
        try:
            for i in range(reps):
                if before is not None:
                    before()
                L.wtp_set_kernel_stamps(ctypes.c_void_p(base + 16 * i))
                step() if not sharded else compute()
        finally:
            L.wtp_set_kernel_stamps(None)
        torch.cuda.synchronize()
        h = st.cpu().numpy().view(np.uint64)
        return (h[:, 1] - h[:, 0]).astype(np.float64) * 0.01  # 100 MHz ticks -> us

    stage_us, dom, dom_us, dom_bytes, dom_launches, timing_src = {}, None, None, 0, 1, None
    work = None
    if (resident or small) and xs:
        # one launch per step: its algorithmic bytes are every weight read once and written once
        spans = stamp_spans(args.stamp_reps)
        dom = "k_resident" if resident else "k_small"
        dom_us, dom_bytes = float(np.mean(spans)), 8 * n_w
        timing_src = ("in-kernel s_memrealtime stamps: first workgroup start -> last workgroup end after its "
                      "stores completed, mean of %d back-to-back launches (wtp_set_kernel_stamps)" % len(spans))
        stage_us = {dom: dom_us}
    elif xs and args.stage_reps > 0:
        # stage intervals from HIP events the library records between its launches (include dispatch
        # gaps); a spin kernel in front lets the whole call be enqueued before it runs
        sevs = [torch.cuda.Event(enable_timing=True) for _ in range(len(STAGES) + 1)]
        for e in sevs:
            e.record()
        torch.cuda.synchronize()
        handles = (ctypes.c_void_p * len(sevs))(*[e.cuda_event for e in sevs])
        per_st = {st: [] for st in STAGES}
        L.wtp_set_stage_events(handles, len(sevs))
        # the stage intervals need the stages in sequence on one stream: the selection pipeline
        # (wtp_set_pipeline, several launch groups) is switched off for this leg only
        pipe_prev = engine.set_pipeline(False)
        try:
            for _ in range(args.stage_reps):
                torch.cuda._sleep(1_000_000)
                step() if not sharded else compute()
                torch.cuda.synchronize()
                for i, st in enumerate(STAGES):
                    per_st[st].append(sevs[i].elapsed_time(sevs[i + 1]) * 1e3)
        finally:
            L.wtp_set_stage_events(None, 0)
            engine.set_pipeline(pipe_prev)

        work = None if args.flatten else dwt_stage_work(
            [(tuple(x.shape), r["eff_level"]) for x, r in zip(xs, recs)], int(L.wtp_dec_len(engine.wavelet_id(wavelet))))

        def sbytes(st):
            if st in DWT_STAGES and not has_dwt:
                return 0
            if st in DWT_STAGES and work is not None:
                return work[st]  # the stage kernels' own inputs and outputs, level by level
            return {"forward_dwt": 4 * n_w + 4 * pop, "k_window": 0, "k_collect": 4 * pop,
                    "k_mask_select": 8 * n_w if pop == n_w else 0, "inverse_dwt": 4 * pop + 4 * n_w}[st]
        ran = [st for st in STAGES if not (st in DWT_STAGES and not has_dwt)]
        stage_us = {st: float(np.median(per_st[st])) for st in ran}
        dom = max((st for st in ran if sbytes(st) > 0), key=lambda st: stage_us[st])
        dom_us, dom_bytes = stage_us[dom], sbytes(dom)
        dom_launches = max(r["eff_level"] for r in recs) if dom in DWT_STAGES else 1
        timing_src = ("HIP events around the stage on the library's stream (median of %d calls, selection "
                      "pipeline off; the interval includes dispatch gaps)" % args.stage_reps)
    dom_kernel = dom if dom in ("k_resident", "k_small") else KERNEL_OF_STAGE.get(dom, dom)
    if dom_us is not None and dom_us > ms_per_step * 1e3 and world == 1:
        timing_src += "; capped at ms_per_step"
        dom_us = ms_per_step * 1e3
    traffic, traffic_src, traffic_tag = pmc_traffic(args.config, dom_kernel) if dom else (None, None, None)
    stamps_us = dom_us if dom in ("k_resident", "k_small") else None
    prof_ns, prof_calls = rocprof_kernel(prof_stats, dom_kernel) if dom else (0.0, 0)
    if prof_calls:
        # the durations rocprofv3 records for the dominant kernel in the child run of this
        # configuration (dispatch to completion, what profiles/ summaries hold), per step: a
        # stage's launches (levels x image groups) summed
        nsteps = child_steps(args)
        dom_launches = prof_calls / nsteps
        dom_us = prof_ns / nsteps * 1e-3
        timing_src = ("rocprofv3 --kernel-trace --stats of this configuration's step loop, run as a child of "
                      "this bench: %d launches of %s over %d steps, device time per step"
                      % (prof_calls, dom_kernel, nsteps))

    # ------------------------------------------------ cold Infinity Cache (MALL)
    # two cold states: "write" -- a 512 MiB write to another buffer between steps, which leaves the
    # 256 MiB Infinity Cache full of that buffer's DIRTY lines (every line the step brings in first
    # writes one of them back to HBM); "read" -- a 512 MiB read of another buffer, which leaves it
    # full of clean lines (the step's data comes from HBM, nothing else is written back)
    cold = None
    if not args.no_cold and not sharded and xs:
        flush = torch.empty(512 << 20 >> 2, dtype=torch.float32, device=dev)
        flush.fill_(1.0)
        cold = {}
        for kind, fl in (("write", lambda: flush.fill_(1.0)), ("read", lambda: flush.sum())):
            cev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.cold_reps)]
            for a, b in cev:
                fl()
                a.record()
                step()
                b.record()
            torch.cuda.synchronize()
            cms = np.array([a.elapsed_time(b) for a, b in cev])
            c = {"ms_per_step_p50": float(np.median(cms)), "ms_per_step_p10": float(np.percentile(cms, 10)),
                 "ms_per_step_p90": float(np.percentile(cms, 90)), "reps": len(cev),
                 "note": ("a 512 MiB %s of another buffer between steps evicts the 256 MiB Infinity Cache "
                          "(%s); eager launches, per-step HIP events (include the launch's dispatch gap)"
                          % (kind, "leaving it full of dirty lines" if kind == "write" else "clean lines"))}
            if resident or small:
                cspans = stamp_spans(args.cold_reps, before=fl)
                cus = float(np.mean(cspans))
                c[dom + "_us"] = cus
                c["roofline_frac"] = dom_bytes / (cus * 1e-6) / 1e9 / HBM_PEAK_GBS
            if kind == "write":
                cold.update(c)
            else:
                cold["after_read_flush"] = c
        del flush

    # ------------------------------------------------- N > 1 legs (cfg4 split, replicas)
    multi = None
    if sharded:
        Kc = max(20, K // 4)
        t_comp = timed(Kc, compute) / Kc * 1e3
        t_gath = timed(Kc, gather) / Kc * 1e3
        rep_outs = [torch.empty_like(x) for x in xs_all]
        rep_res = torch.empty(len(xs_all) * REC_BYTES, dtype=torch.uint8, device=dev)

        def replica():
            engine.launch(xs_all, wavelet, level, pct, outs=rep_outs, carry_level=False, results=rep_res)
        for _ in range(3):
            replica()
        t_rep = timed(Kc, replica) / Kc * 1e3
        xname = "batch_isend_irecv" if args.exchange == "p2p" else "all_gather_into_tensor"
        multi = {"cfg4_one_model": {"exchange": args.exchange, "end_to_end_ms": ms_per_step, "compute_ms_max_rank": t_comp,
                                    "all_gather_ms": t_gath, "max_rank_weights": int(plan.max_shard),
                                    "bytes_sent_this_rank": plan.bytes_sent(rank),
                                    "bytes_received_this_rank": plan.bytes_received(rank),
                                    "bytes_received_max_rank": max(plan.bytes_received(r) for r in range(world)),
                                    "largest_region_bytes": 4 * max(plan.size),
                                    "per_link_estimate_us": (4 * max(plan.size) / XGMI_LINK_GBS / 1e3 if args.exchange == "p2p"
                                                             else 4 * plan.stride * (world - 1) / XGMI_LINK_GBS / 1e3),
                                    "exchange_status": (("rehearsal: %s over %s with every rank on one "
                                                         "GPU, a functional check; RCCL at N > 1 is not measured by "
                                                         "this line" % (xname, dist.get_backend())) if rehearsal else
                                                        ("%s over %s (RCCL on ROCm) across %d GPUs, "
                                                         "measured by this line" % (xname, dist.get_backend(), world))),
                                    "per_link_estimate_note": ("assumes every peer pair on its own xGMI link at %.0f "
                                                               "GB/s, the largest region the longest copy" % XGMI_LINK_GBS
                                                               if args.exchange == "p2p" else
                                                               "ring all-gather: (N - 1) padded regions through one "
                                                               "xGMI link at %.0f GB/s" % XGMI_LINK_GBS),
                                    "note": ("LPT layer shards pruned in place into the flat state_dict buffer, then "
                                             + ("ONE full-mesh exchange of the unpadded regions (weights + records; "
                                                "batch_isend_irecv = one RCCL group of point-to-point copies, one per "
                                                "xGMI peer link)" if args.exchange == "p2p" else
                                                "ONE in-place all_gather_into_tensor of the regions padded to the "
                                                "largest (weights + records)") + "; eager launches")},
                 "replicas": {"value": world * n_model / (t_rep * 1e-3), "ms_per_step": t_rep, "scaling": "weak",
                              "note": "every rank prunes its own full model, no collective"}}

    # --------------------------------------------- CPU baseline (rank 0, N = 1 only)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import oracle as O
        host = [O.synth(s, seed, tid, e) for (s, seed, tid, e) in mine]
        if args.config == "cfg5":
            host = host[:2]  # bounded sample: two 4096^2 blocks
        n_host = sum(h.size for h in host)

        def leg(nthreads, seconds):
            O.prune_batch(host[:1], wavelet, level, pct, nthreads=nthreads)
            reps, t0 = 0, time.perf_counter()
            while True:
                O.prune_batch(host, wavelet, level, pct, nthreads=nthreads)
                reps += 1
                if time.perf_counter() - t0 >= seconds:
                    break
            return reps, time.perf_counter() - t0
        nt = min(cpu_threads(), O.max_threads())
        r1, t1 = leg(1, args.cpu_seconds / 2)
        rn, tn = leg(nt, args.cpu_seconds / 2)
        try:
            import pywt  # noqa: F401
            pywt_note = "importable (not timed: third-party, not the reference)"
        except Exception as exc:
            pywt_note = "unavailable on this host (%s): the reference's PyWavelets path cannot run here" % type(exc).__name__
        cpu = {"value": n_host * rn / tn, "unit": "weight-coeffs/s", "cores": nt, "kind": "port",
               "cpu_model": cpu_model(), "pywt": pywt_note,
               "sample": "%d passes over %d weights of the %s workload with the C restatement "
                         "(oracle/wtprune_oracle.c, OpenMP over tensors, %d threads), %.1f s"
                         % (rn, n_host, name, nt, tn),
               "single_thread": {"value": n_host * r1 / t1, "cores": 1,
                                 "sample": "%d passes, %.1f s (the reference's execution model: one thread)"
                                           % (r1, t1)}}

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "weight-coeffs/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong" if world > 1 else "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (splitmix64 Irwin-Hall, kaiming-scaled)",
            "config": {"workload": name, "config": args.config if not sharded else "cfg4",
                       "wavelet": wavelet, "level": level, "percentile": pct, "weights_per_step": n_model,
                       "weights_this_rank": n_w, "coeffs_this_rank": pop, "tensors": len(model),
                       "eff_levels": sorted({r["eff_level"] for r in recs}),
                       "graph_steps": G if graph is not None else 0,
                       "parallelism": ("lpt-layer-shard%d+%s" % (world, "allgather-p2p" if args.exchange == "p2p"
                                                                 else "allgather-ring") if sharded
                                       else ("block-split%d" % world if world > 1 else "single")),
                       "transform": "1-D flattened (extension)" if args.flatten else "2-D over (kh, kw) (reference)",
                       # wtp_set_fused_select: launch groups of large DWT tensors (cfg5) take their window
                       # from input patches before the forward and never re-read P for the selection
                       # (the stage leg's "k_collect" is then k_fslot_collect, its "forward_dwt" includes k_fwin)
                       "selection": "window / collect / select over P" if args.no_fused_select
                                    else "fused where a group qualifies (k_fwin, k_fwd_int classification, k_fslot_collect)"},
            "value_source": value_src,
            "timed_region": timed_region,
            "pipeline_hbm_gbs": 8 * n_model / (ms_per_step * 1e-3) / 1e9,
            "step_distribution_ms": dist_ms,
            "roofline": None if dom is None else {
                "bound": "hbm", "kernel": dom_kernel, "stage": dom, "launches_per_stage": dom_launches,
                "achieved": dom_bytes / (dom_us * 1e-6) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": dom_bytes / (dom_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                "traffic": traffic,  # per launch, like achieved (bytes per launch / average launch)
                "traffic_per_step": None if traffic is None else traffic * dom_launches,
                "traffic_source": traffic_src and ("committed rocprofv3 --pmc summary %s (2 x FETCH_SIZE + "
                                                   "WRITE_SIZE per launch), not measured in this run" % traffic_src),
                "algorithmic_bytes_per_step": dom_bytes,
                "algorithmic_bytes_per_launch": dom_bytes / max(dom_launches, 1),
                "bytes_basis": ("every weight read once and written once (8 B per weight)" if dom in ("k_resident", "k_small")
                                else "the stage kernels' own inputs and outputs, level by level (tools: dwt_stage_work)"
                                if dom in DWT_STAGES and work is not None else "stage inputs and outputs"),
                "valu_frac": (work["flops_per_stage"] / (dom_us * 1e-6) / (VALU_NOFMA_TFLOPS * 1e12)
                              if dom in DWT_STAGES and work is not None else None),
                "avg_launch_us": dom_us / max(dom_launches, 1), "us_per_step": dom_us, "timing": timing_src,
                "avg_launch_us_stamps": stamps_us, "pmc_source_tag": traffic_tag},
            "stage_us": stage_us,
            "cpu_baseline": cpu,
        }
        if faults:
            line["resident_faults"] = faults
        if faults_timed:
            line["resident_faults_timed"] = faults_timed
            line["valid"] = False  # a timed step hit the resident timeout: this line is not a measurement
        if args.config == "cfg5":
            flops = DB8_L5_FLOP_PER_ELEM * n_model
            line["valu_roof"] = {"flop_per_elem": DB8_L5_FLOP_PER_ELEM, "peak_tflops": VALU_NOFMA_TFLOPS,
                                 "floor_ms": flops / (VALU_NOFMA_TFLOPS * 1e12) * 1e3 / world,
                                 "frac": flops / (ms_per_step * 1e-3) / (VALU_NOFMA_TFLOPS * 1e12) / world,
                                 "note": "whole pipeline vs the no-FMA FP32 VALU rate measured on MI355X "
                                         "(bit-exactness forbids contraction); the dominant kernel's own "
                                         "fraction is roofline.valu_frac"}
        if cold:
            line["cold_mall"] = cold
        if multi:
            line.update(multi)
        if rehearsal and world > 1:
            line["rehearsal"] = "all ranks on one GPU over gloo: a functional check, not a measurement"
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
