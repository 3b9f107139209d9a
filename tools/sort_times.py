"""Per-workgroup sort timing probe (tmp_ab/t_sorttime build, blend disabled):
each sort workgroup writes (start, end, list length, class) into rgba[blockIdx]."""
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
u = rgba.reshape(-1, 4).view(np.uint32)
nt = s_ntiles if False else None
nwg = int(os.environ.get('NWG', '10200'))
u = u[:nwg]
t0, t1, L, C = [u[:, i].astype(np.int64) for i in range(4)]
ok = t1 > 0
t0, t1, L, C = t0[ok], t1[ok], L[ok], C[ok]
base = t0.min(); t0 -= base; t1 -= base
print("workgroups", ok.sum(), "span us", t1.max() / 100)
for c, name in ((2, "medium"), (1, "small")):
    sel = C == c
    d = (t1 - t0)[sel] * 10 / 1000
    print(name, sel.sum(), "dur us pctl 10/50/90/max", np.percentile(d, [10, 50, 90, 100]) if sel.any() else None,
          "start range", t0[sel].min() / 100 if sel.any() else None, t0[sel].max() / 100 if sel.any() else None,
          "end max", t1[sel].max() / 100 if sel.any() else None)
sel = C == 2
if sel.any():
    for lo, hi in ((256, 512), (512, 768), (768, 1024), (1024, 1536), (1536, 2048)):
        m = sel & (L > lo) & (L <= hi)
        if m.any():
            print(f"  medium L in ({lo},{hi}]: n={m.sum()} mean dur us {((t1 - t0)[m] * 10 / 1000).mean():.2f}")
tt = np.arange(0, t1.max() / 100 + 1, 2.0)
print("live WGs over time:", [int(((t0 / 100 <= t) & (t1 / 100 > t)).sum()) for t in tt])
# phase split of the medium sorts (t_sortphase build: column 3 holds the
# timestamp after the register bitonic runs instead of the class)
u2 = rgba.reshape(-1, 4).view(np.uint32)[:nwg]
tb = u2[:, 3].astype(np.int64)
med = (tb > 1000) & ok
if med.any():
    s0 = u2[med, 0].astype(np.int64); s1 = u2[med, 1].astype(np.int64); sb = tb[med]
    print("medium phase us: bitonic (load+sort) mean", ((sb - s0) * 10 / 1000).mean(), " merge+store mean", ((s1 - sb) * 10 / 1000).mean())
