"""d/dpts mask-only backward of one library build, saved for a bit-for-bit comparison with another
(NSLAM_LIB=... python tools/probes/pg_equal.py OUT.npz): the tiny scene's frames, 600 rays, the colour
stage's three decoders, random cotangent; saves every decoder's d/dpts share and the grid gradients."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import conftest  # noqa: E402
import test_gpu_fused as T  # noqa: E402

with np.load(os.path.join(conftest.GOLDEN, "tiny_scene.npz")) as z:
    tiny = {k: z[k] for k in z.files}
sc, frames = T._frames(tiny)
nice, c = T._nice(sc)
eng = T.P.engine.MappingEngine(nice, c, sc.bound, 32, 16, device=T.DEV)
g = torch.Generator(device=T.DEV).manual_seed(7)
pix = torch.randint(96 * 128, (600,), device=T.DEV, generator=g)
ro, rd, gd, gc, keep = T.P.ops.gather_rays(frames[:1], pix, 600, 96, 128, (0, 96, 0, 128), sc.fx, sc.fy, sc.cx, sc.cy)
z = T.P.ops.sample_z(ro, rd, gd, sc.bound, 32, 16)
eng.query_fwd("color", ro, rd, z)
g_raw = torch.randn(z.numel(), 4, device=T.DEV, generator=g)
keys = ("grid_middle", "grid_fine", "grid_color")
eng.gall.zero_()
parts = eng.query_bwd("color", ro, rd, z, g_raw, keys, (), pts_grad=True, pts_parts=True)
torch.cuda.synchronize()
np.savez(sys.argv[1], **{f"gp{i}": p.cpu().numpy() for i, p in enumerate(parts)},
         **{k: eng.ggrad[k].cpu().numpy() for k in keys})
print("saved", sys.argv[1], [p.shape for p in parts])
