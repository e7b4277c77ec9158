"""Which small torch ops of the drop-ins' per-call setup can be captured in a hipGraph on this image
(ROCm): torch.linalg.inv_ex on one / a batch of 4x4 poses, torch.randint on the default generator.
Each case captures, replays with new inputs and compares with the eager result."""
import torch

dev = torch.device("cuda:0")
g0 = torch.Generator(device=dev).manual_seed(0)


def case(name, make, fn):
    x = make()
    ref_out = fn(x)  # eager warm-up (handles, workspaces)
    out = torch.empty_like(ref_out)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out.copy_(fn(x))
        ok = True
        for _ in range(3):
            x.copy_(make())
            g.replay()
            torch.cuda.synchronize()
            ok &= bool(torch.equal(out, fn(x)))
        print(f"{name}: captured, replays equal eager: {ok}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{name}: NOT capturable: {type(e).__name__}: {str(e)[:200]}", flush=True)


def pose():
    q = torch.randn(4, device=dev, generator=g0)
    q = q / q.norm()
    w, x, y, z = q
    R = torch.stack([torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)]),
                     torch.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)]),
                     torch.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)])])
    m = torch.eye(4, device=dev)
    m[:3, :3] = R
    m[:3, 3] = torch.randn(3, device=dev, generator=g0)
    return m


case("inv_ex 4x4", pose, lambda a: torch.linalg.inv_ex(a)[0])
case("inv_ex batch 5x4x4", lambda: torch.stack([pose() for _ in range(5)]), lambda a: torch.linalg.inv_ex(a)[0])
case("inverse 4x4", pose, lambda a: a.inverse())
case("matmul chain", pose, lambda a: a @ torch.linalg.inv_ex(a)[0] @ a)
out = torch.empty(100, dtype=torch.int64, device=dev)
g = torch.cuda.CUDAGraph()
try:
    torch.randint(1000, (100,), device=dev)
    with torch.cuda.graph(g):
        out.copy_(torch.randint(1000, (100,), device=dev))
    g.replay()
    a = out.clone()
    g.replay()
    print("randint default generator: captured, fresh draws per replay:", not torch.equal(a, out), flush=True)
except Exception as e:  # noqa: BLE001
    print(f"randint: NOT capturable: {type(e).__name__}: {str(e)[:200]}", flush=True)
