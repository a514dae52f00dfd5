"""A child process for tests/test_gpu_scenes.py::test_exit_with_live_contexts:
creates a context and a multi context (one device listed twice), renders
through both, streams a few device frames in flight, and leaves WITHOUT
destroying either -- the process's normal exit (interpreter teardown, the
shared libraries' finalizers) must end with status 0.  XRT_SEGV_TRACE=1 in
its environment names the library of any fatal signal."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import simpleraytracing_amd as xrt
    tris = xrt.load_ply(os.path.join(ROOT, "data", "dragon.ply"))
    cam = xrt.camera_for_mesh(tris, 256, 256)
    # leaked on purpose: no close(), no __del__ teardown
    xrt.Context.__del__ = lambda self: None
    xrt.MultiContext.__del__ = lambda self: None
    c = xrt.Context(0)
    c.upload_mesh(tris)
    img, lb, u8, st = c.render_rows(cam)
    m = xrt.MultiContext([0, 0])
    m.upload_mesh(tris)
    got = m.render(cam)
    ok = bool((got[1].view("u4") == lb.view("u4")).all())
    c.render_frames(cam, 6)             # frames through the pinned ring and copy threads
    print("exit job:", "ok" if ok else "MISMATCH", st.hit_rays, flush=True)
    globals()["_keep"] = (c, m)         # both still alive at interpreter exit
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
