"""Which float32 formula does torch's get_rays_from_uv (common.py:74-89) compute on the device?"""
import torch
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
n = 200000
i = torch.randint(0, 1200, (n,), device=dev, generator=g).float()
j = torch.randint(0, 680, (n,), device=dev, generator=g).float()
c2w = torch.randn(3, 4, device=dev, generator=g)
fx, fy, cx, cy = 600.0, 600.0, 599.5, 339.5
dirs = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1)
ref = torch.sum(dirs.reshape(-1, 1, 3) * c2w[:3, :3], -1)
R = c2w[:3, :3]
for name, d0, d1 in (("recip", (i - cx) * torch.tensor(1.0 / fx, dtype=torch.float32), -(j - cy) * torch.tensor(1.0 / fy, dtype=torch.float32)),
                     ("truediv", (i - cx) / torch.tensor(fx, device=dev), -(j - cy) / torch.tensor(fy, device=dev))):
    print(name, "d0 equal", torch.equal(d0, dirs[:, 0]), "d1 equal", torch.equal(d1, dirs[:, 1]))
p = [dirs[:, None, m] * R[None, :, m] for m in range(3)]  # [n,3] each
for nm, v in (("(p0+p1)+p2", (p[0] + p[1]) + p[2]), ("p0+(p1+p2)", p[0] + (p[1] + p[2])),
              ("(p0+p2)+p1", (p[0] + p[2]) + p[1]), ("fma chain", torch.addcmul(torch.addcmul(p[0], dirs[:, None, 1], R[None, :, 1]), dirs[:, None, 2], R[None, :, 2]))):
    print(nm, "equal", torch.equal(v, ref), "mismatch frac", float((v != ref).float().mean()))
