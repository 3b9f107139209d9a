import os, sys, time
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
import torch
from gaussian_splat_ipu_amd import camera, scene
from gaussian_splat_ipu_amd.splatter import GpuSplatter
from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=100000, seed=1, sh_degree=0)))
W, H = 1920, 1080
fb = TiledFramebuffer(W, H, 16, 16)
view, proj = camera.headless(bb, W, H)
r = GpuSplatter(g, fb, device=0, band_rows=(30, 39), band_pad_rows=9, band_cull=True, write_rgba=False)
r.set_view_wire(view); r.set_projection_wire(proj); r.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
r.execute()
st = torch.cuda.ExternalStream(r.get_stream())
buf = torch.empty(9 * 16 * W * 3 * 4, dtype=torch.uint8, device='cuda')
ev = torch.cuda.Event(); ev2 = torch.cuda.Event()
ev2.record()
K = 2000
def t(name, f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K): f()
    dt = (time.perf_counter() - t0) / K * 1e6
    torch.cuda.synchronize()
    print(f"{name}: {dt:.2f} us", flush=True)
bb_ = 9 * 16 * W * 3
p = buf.data_ptr()
t("execute_async", lambda: r.execute_async())
r.sync()
t("copy_bgr8_device", lambda: r.copy_bgr8_device(p, bb_))
t("event.record(ext stream)", lambda: ev.record(st))
t("stream.wait_event", lambda: st.wait_event(ev2))
comm = torch.cuda.Stream()
def ctx():
    with torch.cuda.stream(comm):
        pass
t("stream context", ctx)
t("set_view_wire", lambda: r.set_view_wire(view))
