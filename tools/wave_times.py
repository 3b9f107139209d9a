"""Per-wave blend timing probe (tmp_ab/t_wavetime build): each wave writes its
s_memrealtime start/end (100 MHz) into its first pixel's R/G; this script
renders the bench frame and prints the wave-duration distribution and the
kernel's tail (how long the last waves run after most have finished)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from gaussian_splat_ipu_amd import camera, scene
from gaussian_splat_ipu_amd.splatter import GpuSplatter
from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
W, H, TW = 1920, 1080, 16
g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=1_000_000, seed=1, sh_degree=3)))
view, proj = camera.headless(bb, W, H)
fb = TiledFramebuffer(W, H, TW, TW)
NB = int(os.environ.get('BANDS', '1'))
with GpuSplatter(g, fb, device=0, band_index=min(2, NB - 1), band_count=NB, band_interleaved=NB > 1, band_cull=NB > 1) as s:
    s.set_view_wire(view); s.set_projection_wire(proj); s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
    for _ in range(5):
        s.execute()
    rgba = s.get_rgba()
u = rgba.view(np.uint32)
# first pixel of each 8x8 block
blk = u[0::8, 0::8]  # [H/8, W/8, 4]
blk = blk[(blk[..., 1] != 0)]  # rows this band rendered (1-D list of waves)
t0 = blk[..., 0].astype(np.int64); t1 = blk[..., 1].astype(np.int64)
base = t0.min()
t0 -= base; t1 -= base
d = (t1 - t0) * 10  # ns
print("waves", d.size, "kernel span us", (t1.max()) / 100.0)
print("wave duration us pctl 10/50/90/99/max", np.percentile(d, [10, 50, 90, 99, 100]) / 1000)
ends = np.sort(t1.ravel()) / 100.0
print("end time us at fraction 0.5/0.9/0.99/1.0:", [ends[int(f * (ends.size - 1))] for f in (0.5, 0.9, 0.99, 1.0)])
starts = np.sort(t0.ravel()) / 100.0
print("start time us at fraction 0.25/0.5/0.9/1.0:", [starts[int(f * (starts.size - 1))] for f in (0.25, 0.5, 0.9, 1.0)])
np.save("gpurun_out/wave_times.npy", np.stack([t0, t1]))
tt = np.arange(0, t1.max() / 100.0 + 1, 2.0)
print("live waves over time (2 us steps):", [int(((t0 / 100.0 <= t) & (t1 / 100.0 > t)).sum()) for t in tt])
print("mean live waves over the span:", ((t1 - t0).sum() / 100.0) / (t1.max() / 100.0))
# duration map, coarse
dm = (d / 1000.0)

nb = blk[..., 2].astype(np.int64)
it = blk[..., 3].astype(np.int64)
if not it.any():
    raise SystemExit(0)
mi, su = it & 0xFFF, it >> 12
print("batches per wave pctl 50/90/max", np.percentile(nb, [50, 90, 100]))
print("max-lane iterations per wave pctl 50/90/max", np.percentile(mi, [50, 90, 100]), "total", mi.sum())
print("lane-iteration efficiency (sum/64/max)", su.sum() / 64 / mi.sum())
sel = d > 20000
print("heavy waves (>20us):", sel.sum(), "mean batches", nb[sel].mean(), "mean max-iters", mi[sel].mean(), "mean dur us", d[sel].mean() / 1000)
sel = d < 8000
print("light waves (<8us):", sel.sum(), "mean batches", nb[sel].mean(), "mean max-iters", mi[sel].mean(), "mean dur us", d[sel].mean() / 1000)
