"""Calibrate the synthetic scene's log-scale mean (SURVEY §8 d): median
projected radius ~4 px at 1920x1080 with fxy[1] = 1 on the headless camera.
Uses the CPU oracle's projection (test infrastructure).  Result (round 1):
mu = -5.6  ->  radius p10/p50/p90/p99 = 3/4/6-7/9-11 px."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gaussian_splat_ipu_amd import camera, scene  # noqa: E402
from oracle import oracle as O  # noqa: E402

for mu in [-6.0, -5.8, -5.6, -5.4, -5.0]:
    g, bb = scene.prepare_scene(scene.synthetic(scene.SynthSpec(n=100000, seed=1, sh_degree=0, log_scale_mu=mu)))
    v, p = camera.headless(bb, 1920, 1080)
    f = O.make_frame(v, p, 1920, 1080, 16, 16, camera.FOV_DEFAULT, 1.0)
    pr = O.project(g, f)
    r = pr["radius"][pr["rendered"] != 0]
    print(f"mu={mu:5.2f} radius p10/p50/p90/p99 = {np.percentile(r, [10, 50, 90, 99])}")
