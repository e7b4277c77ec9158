"""CPU emulation of the kernels' MFMA tile algebra over the PACKED decoder buffers.

v_mfma_f32_32x32x2_f32 semantics used by csrc/nslam_query.hip (CDNA4 guide §3):
  A operand: lane l holds A[i=l&31][k=l>>5];  B operand: lane l holds B[k=l>>5][j=l&31]
  C/D: lane l holds column j=l&31, register r holds row F(r, l>>5).
This test runs the same chaining (tile register s == B operand of step s) with numpy on the
packed index maps and compares with a direct numpy MLP, so a wrong index map fails on CPU.
"""
import numpy as np
import pytest
import torch

F = lambda r, h: (r & 3) + 8 * (r >> 2) + 4 * h  # noqa: E731
LANE = np.arange(64)


def to_tile(X):
    """X [32 features][32 points] → tile [64 lanes][16 regs]."""
    t = np.empty((64, 16))
    for l in range(64):
        for r in range(16):
            t[l, r] = X[F(r, l >> 5), l & 31]
    return t


def from_tile(t):
    X = np.empty((32, 32))
    for l in range(64):
        for r in range(16):
            X[F(r, l >> 5), l & 31] = t[l, r]
    return X


def gemm_acc(acc, frag, x):
    """acc (tile) += A(frag) * B(x tile), 16 steps of 32x32x2."""
    D = from_tile(acc)
    fr = frag.reshape(64, 16)
    for s in range(16):
        A = np.stack([fr[:32, s], fr[32:, s]], 1)          # [32 i][2 kk]
        B = np.stack([x[:32, s], x[32:, s]], 0)             # [2 kk][32 j]
        D = D + A @ B
    return to_tile(D)


def vec_tile(v):
    return to_tile(np.repeat(np.asarray(v)[:, None], 32, 1))


def packed_numpy(packer, module):
    flat = np.concatenate([p.detach().numpy().reshape(-1) for p in module.parameters()] + [np.zeros(1)])
    idx = np.where(packer.index >= 0, packer.index, packer.n_params)
    return flat[idx]


@pytest.fixture(scope="module")
def nice(pkg):
    torch.manual_seed(0)
    return pkg.NICE(c_dim=32, coarse=True, hidden_size=32, coarse_grid_len=2.0, middle_grid_len=0.32)


@pytest.mark.parametrize("name", ["middle", "fine", "color"])
def test_xyz_forward_and_transposed_blocks(nice, name):
    dec = nice.decoder(name)
    pk_ = dec.packer()
    pk = packed_numpy(pk_, dec)
    L = pk_.layout
    FR = 1024
    rng = np.random.default_rng(1)
    nc = 2 if name == "fine" else 1
    x = rng.normal(size=(32, 3)).astype(np.float64)            # 32 points
    cin = [rng.normal(size=(32, 32)) for _ in range(nc)]        # [feat][pt] per block
    sd = {k: v.detach().numpy().astype(np.float64) for k, v in dec.state_dict().items()}
    # reference MLP (points as rows)
    emb = np.sin(x @ sd["embedder._B"])
    feat = np.concatenate([c.T for c in cin], 1)
    h = emb
    for i in range(5):
        h = np.maximum(h @ sd[f"pts_linears.{i}.weight"].T + sd[f"pts_linears.{i}.bias"], 0) \
            + feat @ sd[f"fc_c.{i}.weight"].T + sd[f"fc_c.{i}.bias"]
        if i == 2:
            h = np.concatenate([emb, h], 1)
    out_ref = h @ sd["output_linear.weight"].T + sd["output_linear.bias"]

    # emulated kernel (xyz_forward in nslam_query.hip)
    B = pk[L["FB"]:L["FB"] + 288].reshape(3, 96)
    e_full = np.sin(x @ B)                                     # [32 pts][96]
    e = [to_tile(e_full[:, 32 * b:32 * b + 32].T) for b in range(3)]
    ct = [to_tile(c) for c in cin]
    blk = lambda j: pk[j * FR:(j + 1) * FR]  # noqa: E731

    def fc(i):
        z = vec_tile(pk[L["BiasC"] + 32 * i:L["BiasC"] + 32 * i + 32])
        for c in range(nc):
            z = gemm_acc(z, blk(L[f"FC{i}_{c}"]), ct[c])
        return z

    a = vec_tile(pk[L["Bias"]:L["Bias"] + 32])
    a3 = vec_tile(pk[L["Bias"] + 96:L["Bias"] + 128])
    for b in range(3):
        a = gemm_acc(a, blk(L["L0"] + b), e[b])
        a3 = gemm_acc(a3, blk(L["L3"] + b), e[b])
    hh = np.maximum(a, 0) + fc(0)
    for i, key in ((1, "L1"), (2, "L2")):
        a = gemm_acc(vec_tile(pk[L["Bias"] + 32 * i:L["Bias"] + 32 * i + 32]), blk(L[key]), hh)
        hh = np.maximum(a, 0) + fc(i)
    a3 = gemm_acc(a3, blk(L["L3"] + 3), hh)
    hh = np.maximum(a3, 0) + fc(3)
    a = gemm_acc(vec_tile(pk[L["Bias"] + 128:L["Bias"] + 160]), blk(L["L4"]), hh)
    hh = np.maximum(a, 0) + fc(4)
    H4 = from_tile(hh)                                          # [32 feat][32 pts]
    nout = 4 if name == "color" else 1
    Wo = pk[L["Wo"]:L["Wo"] + 128].reshape(4, 32)[:nout]
    out = (Wo @ H4).T + pk[L["Bo"]:L["Bo"] + nout]
    np.testing.assert_allclose(out, out_ref, rtol=1e-9, atol=1e-9)

    # transposed blocks: W^T * dY for layer 4 and the 4 blocks of layer 3
    dY = rng.normal(size=(32, 32))
    got = from_tile(gemm_acc(np.zeros((64, 16)), blk(L["L4T"]), to_tile(dY)))
    np.testing.assert_allclose(got, sd["pts_linears.4.weight"].T @ dY, rtol=1e-9, atol=1e-9)
    W3 = sd["pts_linears.3.weight"]
    W3pad = np.zeros((32, 128))
    W3pad[:, :93] = W3[:, :93]
    W3pad[:, 96:] = W3[:, 93:]
    for b in range(4):
        got = from_tile(gemm_acc(np.zeros((64, 16)), blk(L["L3T"] + b), to_tile(dY)))
        np.testing.assert_allclose(got, W3pad[:, 32 * b:32 * b + 32].T @ dY, rtol=1e-9, atol=1e-9)
    got = from_tile(gemm_acc(np.zeros((64, 16)), blk(L["FCT2"]), to_tile(dY)))
    np.testing.assert_allclose(got, sd["fc_c.2.weight"][:, :32].T @ dY, rtol=1e-9, atol=1e-9)


def test_coarse_forward(nice):
    dec = nice.decoder("coarse")
    pk_ = dec.packer()
    pk = packed_numpy(pk_, dec)
    L = pk_.layout
    FR = 1024
    blk = lambda j: pk[j * FR:(j + 1) * FR]  # noqa: E731
    sd = {k: v.detach().numpy().astype(np.float64) for k, v in dec.state_dict().items()}
    c = np.random.default_rng(2).normal(size=(32, 32))  # [feat][pt]
    h = c.T
    for i in range(5):
        h = np.maximum(h @ sd[f"pts_linears.{i}.weight"].T + sd[f"pts_linears.{i}.bias"], 0)
        if i == 2:
            h = np.concatenate([c.T, h], 1)
    ref = h @ sd["output_linear.weight"].T + sd["output_linear.bias"]
    ct = to_tile(c)
    bias = lambda i: vec_tile(pk[L["Bias"] + 32 * i:L["Bias"] + 32 * i + 32])  # noqa: E731
    a = gemm_acc(bias(0), blk(L["L0"]), ct)
    a3 = gemm_acc(bias(3), blk(L["L3"]), ct)
    hh = np.maximum(a, 0)
    hh = np.maximum(gemm_acc(bias(1), blk(L["L1"]), hh), 0)
    hh = np.maximum(gemm_acc(bias(2), blk(L["L2"]), hh), 0)
    hh = np.maximum(gemm_acc(a3, blk(L["L3"] + 1), hh), 0)
    hh = np.maximum(gemm_acc(bias(4), blk(L["L4"]), hh), 0)
    out = (pk[L["Wo"]:L["Wo"] + 32] @ from_tile(hh)) + pk[L["Bo"]]
    np.testing.assert_allclose(out, ref[:, 0], rtol=1e-9, atol=1e-9)
