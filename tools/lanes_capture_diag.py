"""Lab: which form of the per-group lane streams (wtp_set_pipeline(2)) crashes at graph capture
end.  Each variant runs in a child process (a crash ends only that child): prints rc per variant.
Usage: python tools/lanes_capture_diag.py            (runs every variant)
       python tools/lanes_capture_diag.py VARIANT    (one variant, in this process)"""
import faulthandler
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SHAPES = [(2, 3, 64, 64), (1, 1, 130, 97), (3, 2, 33, 40), (1, 4, 128, 128)] * 12 + [(16, 8, 1, 1), (2, 2, 96, 80),
                                                                                     (1, 1, 200, 64)]
# least likely to crash first: the runner stops at the first variant that fails (after a crash no
# further GPU work is started in the same call)
# measured (round 5, profiles/r05_lanes_capture.txt): torch_lane_to_lane and torch_hub pass,
# torch_side_lane_cross segfaults in capture_end (run it by name, last: nothing may follow a crash);
# the library's lanes (relayed through the caller's stream) pass
VARIANTS = ["torch_lane_to_lane", "torch_hub", "lanes_prewarmed_stream", "lanes_1call", "lanes_3calls"]


def run(v):
    faulthandler.enable()
    import torch
    if v == "pure_torch_4streams":
        x = torch.ones(1 << 20, device="cuda")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cap = torch.cuda.current_stream()
            fork = torch.cuda.Event()
            fork.record(cap)
            lanes = [torch.cuda.Stream() for _ in range(4)]
            outs = []
            for i, l in enumerate(lanes):
                l.wait_event(fork)
                with torch.cuda.stream(l):
                    outs.append(x * (i + 1))
            for l in lanes:
                e = torch.cuda.Event()
                e.record(l)
                cap.wait_event(e)
        g.replay()
        torch.cuda.synchronize()
        return
    if v == "torch_hub":
        # the same dependencies routed through the captured stream: forked streams wait only on
        # events recorded on it, and it waits on theirs
        x = torch.ones(1 << 20, device="cuda")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cap = torch.cuda.current_stream()

            def hub(from_stream):
                e = torch.cuda.Event()
                e.record(from_stream)
                cap.wait_event(e)
                h = torch.cuda.Event()
                h.record(cap)
                return h
            fork = torch.cuda.Event()
            fork.record(cap)
            lanes = [torch.cuda.Stream() for _ in range(3)]
            side = torch.cuda.Stream()
            side.wait_event(fork)
            outs = []
            for i, l in enumerate(lanes):
                l.wait_event(fork)
                with torch.cuda.stream(l):
                    outs.append(x * (i + 1))
                side.wait_event(hub(l))
                with torch.cuda.stream(side):
                    outs.append(x + i)
                l.wait_event(hub(side))
                with torch.cuda.stream(l):
                    outs.append(x - i)
            for l in lanes + [side]:
                e = torch.cuda.Event()
                e.record(l)
                cap.wait_event(e)
        g.replay()
        torch.cuda.synchronize()
        return
    if v.startswith("torch_"):
        # the lanes' dependency graph with trivial kernels: lane_to_lane = a lane waits on an event
        # recorded on another lane (the stagger); side_lane_cross = the side stream waits on a lane's
        # event and the lane on the side stream's; full_topology = both, as wtp_set_pipeline(2) issues
        x = torch.ones(1 << 20, device="cuda")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cap = torch.cuda.current_stream()
            fork = torch.cuda.Event()
            fork.record(cap)
            n = 3
            lanes = [torch.cuda.Stream() for _ in range(n)]
            side = torch.cuda.Stream()
            side.wait_event(fork)
            outs, prev = [], fork
            for i, l in enumerate(lanes):
                l.wait_event(prev if v != "torch_side_lane_cross" else fork)
                with torch.cuda.stream(l):
                    outs.append(x * (i + 1))
                mark = torch.cuda.Event()
                mark.record(l)
                if v != "torch_side_lane_cross":
                    prev = mark
                if v != "torch_lane_to_lane":
                    side.wait_event(mark)
                    with torch.cuda.stream(side):
                        outs.append(x + i)
                    sd = torch.cuda.Event()
                    sd.record(side)
                    l.wait_event(sd)
                    with torch.cuda.stream(l):
                        outs.append(x - i)
            for l in lanes + [side]:
                e = torch.cuda.Event()
                e.record(l)
                cap.wait_event(e)
        g.replay()
        torch.cuda.synchronize()
        return
    from wavelettransforms_amd import engine
    mode = 1 if v.startswith("side") else 2
    engine.set_pipeline(mode)
    xs = [engine.synth(s, 7, i, 6 + (i % 5)) for i, s in enumerate(SHAPES)]
    outs = [torch.empty_like(x) for x in xs]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        engine.launch(xs, "db8", 3, 60.0, outs=outs, carry_level=False, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    calls = 3 if v == "lanes_3calls" else 1
    g = torch.cuda.CUDAGraph()
    if v in ("lanes_prewarmed_stream", "lanes_eager_then_capture_same_stream"):
        if v == "lanes_eager_then_capture_same_stream":
            with torch.cuda.stream(s):
                engine.launch(xs, "db8", 3, 60.0, outs=outs, carry_level=False, stream=s)
            torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(calls):
                engine.launch(xs, "db8", 3, 60.0, outs=outs, carry_level=False, stream=s)
    else:
        with torch.cuda.graph(g):
            for _ in range(calls):
                engine.launch(xs, "db8", 3, 60.0, outs=outs, carry_level=False)
    g.replay()
    torch.cuda.synchronize()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
        print("ok", sys.argv[1])
    else:
        for v in VARIANTS:
            r = subprocess.run([sys.executable, "-X", "faulthandler", os.path.abspath(__file__), v], capture_output=True,
                               text=True, timeout=240)
            tail = (r.stdout + r.stderr).strip().splitlines()[-3:]
            print("%-40s rc=%d  %s" % (v, r.returncode, " | ".join(t for t in tail if "amdgpu.ids" not in t)[:300]),
                  flush=True)
            if r.returncode != 0:
                sys.exit(1)
