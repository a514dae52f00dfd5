"""Frames in flight: the same steady frame rendered K times on one stream into
one buffer set, then alternating over S streams (each with its own output
planes), so that frame k+1's render can start while frame k's last waves run.
Prints the step of each and checks every buffer set against the one-stream
frame bit for bit.

  python tools/inflight_probe.py [--size W H] [--steps K] [--streams S]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, nargs=2, default=(2048, 2048))
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--streams", nargs="+", default=["1", "2", "3"],
                    help="n = n streams of default priority; np = n streams, the first at high priority")
    ap.add_argument("--tile-mesh", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--curve", type=int, default=0, metavar="N",
                    help="first: N frames on 2 streams straight after setup, the host's per-call times "
                         "(the host waits on the GPU) averaged per 100 frames -- how the step evolves")
    ap.add_argument("--timing", nargs="+", type=int, default=[0],
                    help="0: no timed region; 1: the timed frames inside xrt timing_begin/timing_end as bench.py")
    args = ap.parse_args()
    import torch
    import simpleraytracing_amd as xrt
    from simpleraytracing_amd.scenes import tiled_mesh

    W, H = args.size
    dev = torch.device("cuda", 0)
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    if args.tile_mesh > 1:
        tris = tiled_mesh(tris, args.tile_mesh)
    cam = xrt.camera_for_mesh(tris, W, H)
    ctx = xrt.Context(0)
    ctx.upload_mesh(tris)
    n_max = max(int(s.rstrip("p")) for s in args.streams)
    plain = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(n_max - 1)]
    prio = [torch.cuda.Stream(dev, priority=-1)] + plain[1:]
    streams = plain
    planes = [(torch.zeros(W * H, dtype=torch.float32, device=dev), torch.zeros(W * H, dtype=torch.float32, device=dev),
               torch.zeros(W * H, dtype=torch.uint8, device=dev)) for _ in range(n_max)]

    def step(k, s):
        img, lb, u8 = planes[k % s]
        ctx.render_rows_device(cam, 0, H, img.data_ptr(), lb.data_ptr(), u8.data_ptr(), streams[k % s].cuda_stream)

    def use(spec):
        streams[:] = prio if spec.endswith("p") else plain
        return int(spec.rstrip("p"))

    def run(s, n):
        for k in range(n):
            step(k, s)

    if args.curve:
        # three runs: straight after setup, straight after a synchronize, and
        # after a synchronize and 20 ms of host sleep (the GPU idle)
        for idle_ms in (None, 0.0, 20.0):
            torch.cuda.synchronize(dev)
            if idle_ms:
                time.sleep(idle_ms / 1e3)
            stamps = [time.perf_counter()]
            for k in range(args.curve):
                step(k, 2)
                stamps.append(time.perf_counter())
            per = [(stamps[i + 100] - stamps[i]) / 100 * 1e6 for i in range(0, args.curve - 99, 100)]
            print(f"curve (idle before: {idle_ms} ms) us/frame per 100 frames:", " ".join("%.1f" % x for x in per),
                  flush=True)
        torch.cuda.synchronize(dev)
    # the reference frame: one stream, buffer set 0
    run(1, 30)
    torch.cuda.synchronize(dev)
    ref = [t.cpu() for t in planes[0]]
    out = {}
    for rep in range(args.reps):
        for spec, timed in [(a, b) for a in args.streams for b in args.timing]:
            s = use(spec)
            for p in planes:
                for t in p:
                    t.zero_()
            torch.cuda.synchronize(dev)
            run(s, 20 * s)
            torch.cuda.synchronize(dev)
            if timed:
                ctx.timing_begin()
            t0 = time.perf_counter()
            run(s, args.steps)
            torch.cuda.synchronize(dev)
            us = (time.perf_counter() - t0) / args.steps * 1e6
            if timed:
                ctx.timing_end()
            ok = all(torch.equal(planes[b][i].cpu(), ref[i]) for b in range(s) for i in range(3))
            key = spec + ("t" if timed else "")
            out.setdefault(key, []).append(round(us, 2))
            print(f"rep {rep} streams {spec} timing {timed}: step {us:.2f} us  Mrays/s {W * H / us:.0f}  exact {ok}", flush=True)
            if not ok:
                raise SystemExit("frames in flight changed an output")
    print(json.dumps({"size": [W, H], "steps": args.steps, "step_us": out}))


if __name__ == "__main__":
    main()
