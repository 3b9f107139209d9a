"""Host enqueue cost and frames-in-flight throughput of one band of an N-way
split on one GPU (no stage events): python tools/host_launch.py [bands...]"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
from gaussian_splat_ipu_amd import camera, scene
from gaussian_splat_ipu_amd.splatter import GpuSplatter
from gaussian_splat_ipu_amd.tiles import TiledFramebuffer
W, H, TW = 1920, 1080, 16
g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=1_000_000, seed=1, sh_degree=3)))
view, proj = camera.headless(bb, W, H)
fb = TiledFramebuffer(W, H, TW, TW)
for N in [int(v) for v in (sys.argv[1:] or ["1", "8"])]:
    for F in [int(v) for v in os.environ.get('FS', '1,2,3,4').split(',')]:
        R = []
        for f in range(F):
            s = GpuSplatter(g, fb, device=0, band_index=min(2, N - 1), band_count=N, band_interleaved=N > 1,
                            band_cull=N > 1, write_rgba=False,
                            profile=(f == 0 and bool(os.environ.get('PROFILE0'))))
            if f == 0 and os.environ.get('PROFILE0'):
                s.set_profile_interval(1 << 30)
            s.set_view_wire(view); s.set_projection_wire(proj); s.update_focal_lengths(camera.FOV_DEFAULT, 1.0)
            st = None
            if os.environ.get('TORCH_STREAMS'):
                st = torch.cuda.Stream(); s.set_stream(st.cuda_stream)
            s.execute()
            R.append((s, st))
        for k in range(10): R[k % F][0].execute_async()
        torch.cuda.synchronize()
        K = 300
        t0 = time.perf_counter()
        for k in range(K): R[k % F][0].execute_async()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"bands={N} F={F}: host enqueue {1e6*(t1-t0)/K:.1f} us/frame, total {1e6*(t2-t0)/K:.1f} us/frame", flush=True)
        for s, _ in R: s.sync(); s.close()
