"""Decoder weight packing for the fused query kernels.

The MFMA kernels (csrc/nslam_query.hip) read every decoder matrix as 32x32 "fragment blocks":
16 floats per lane, 64 lanes, laid out [lane][step] (one block = 1024 floats = 4 KiB):

  forward block of W[O][K], K-block kb:     frag[l*16+s] = W[l & 31][colmap(kb, F(s, l>>5))]
  transposed block (backward, W^T):         frag[l*16+s] = W[F(s, l>>5)][colmap(kb, l & 31)]
  F(s, h) = (s & 3) + 8*(s >> 2) + 4*h      (the v_mfma_f32_32x32x2_f32 C/D row map)

Packing is ONE device gather `flat_params[index]` per decoder (the index map is built here once
per decoder structure); gradients come back from the kernels in the natural nn.Linear layout
directly into a flat buffer whose offsets are the module's named_parameters order.
The layout constants mirror XyzPack / NoXyzPack in csrc/nslam_dev.h and are cross-checked
against nslam_pack_layout() when the library is present.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

FRAG = 1024
EMB = 93


def F(s, h):
    return (s & 3) + 8 * (s >> 2) + 4 * h


_LANE = np.arange(64)[:, None]
_STEP = np.arange(16)[None, :]
_FIDX = F(_STEP, _LANE >> 5)      # [64,16] feature index of (lane, step)
_COL = np.broadcast_to(_LANE & 31, (64, 16))


def xyz_layout(nc):
    nf = 10 + 5 * nc
    L = {"L0": 0, "L1": 3, "L2": 4, "L3": 5, "L4": 9, "nf": nf,
         "L0T": nf, "L1T": nf + 3, "L2T": nf + 4, "L3T": nf + 5, "L4T": nf + 9, "nfrag": nf + 15}
    for i in range(5):
        for c in range(nc):
            L[f"FC{i}_{c}"] = 10 + i * nc + c
        L[f"FCT{i}"] = nf + 10 + i
    V = L["nfrag"] * FRAG
    L.update(V=V, Bias=V, BiasC=V + 160, Wo=V + 320, Bo=V + 448, FB=V + 452, total=V + 740)
    return L


def noxyz_layout():
    L = {"L0": 0, "L1": 1, "L2": 2, "L3": 3, "L4": 5, "nf": 6,
         "L0T": 6, "L1T": 7, "L2T": 8, "L3T": 9, "L4T": 11, "nfrag": 12}
    V = 12 * FRAG
    L.update(V=V, Bias=V, Wo=V + 160, Bo=V + 288, total=V + 292)
    return L


class DecoderPacker:
    """Index map + gradient offsets for one decoder module (MLP or MLP_no_xyz)."""

    def __init__(self, module, kind: int, nc: int = 1, nout: int = 1):
        self.kind, self.nc, self.nout = kind, nc, nout
        self.names = [n for n, _ in module.named_parameters()]
        self.shapes = {n: tuple(p.shape) for n, p in module.named_parameters()}
        self.offsets = {}
        off = 0
        for n in self.names:
            self.offsets[n] = off
            off += int(np.prod(self.shapes[n]))
        self.n_params = off
        self.layout = xyz_layout(nc) if kind == 0 else noxyz_layout()
        self.index = self._build_index()
        self._dev_index = {}

    # -- index construction ------------------------------------------------------------------
    def _w(self, name):
        return self.offsets[name], self.shapes[name]

    def _frag(self, out, blk, name, colmap, transposed):
        off, (O, K) = self._w(name)
        if transposed:
            o = _FIDX
            k = colmap(_COL)
        else:
            o = _COL
            k = colmap(_FIDX)
        ok = (k >= 0) & (k < K) & (o < O)
        idx = np.where(ok, off + o * K + np.where(k >= 0, k, 0), -1)
        out[blk * FRAG:(blk + 1) * FRAG] = idx.reshape(-1)

    def _vec(self, out, pos, name, length=None):
        off, shp = self._w(name)
        n = int(np.prod(shp))
        out[pos:pos + n] = off + np.arange(n)

    def _build_index(self):
        L = self.layout
        out = np.full(L["total"], -1, dtype=np.int64)
        same = lambda kk: kk  # noqa: E731
        if self.kind == 0:
            pre = ""
            for b in range(3):
                emb_b = lambda kk, b=b: np.where(32 * b + kk < EMB, 32 * b + kk, -1)  # noqa: E731
                self._frag(out, L["L0"] + b, pre + "pts_linears.0.weight", emb_b, False)
                self._frag(out, L["L3"] + b, pre + "pts_linears.3.weight", emb_b, False)
                self._frag(out, L["L0T"] + b, pre + "pts_linears.0.weight", emb_b, True)
                self._frag(out, L["L3T"] + b, pre + "pts_linears.3.weight", emb_b, True)
            h2 = lambda kk: EMB + kk  # noqa: E731
            self._frag(out, L["L3"] + 3, "pts_linears.3.weight", h2, False)
            self._frag(out, L["L3T"] + 3, "pts_linears.3.weight", h2, True)
            for i, key in ((1, "L1"), (2, "L2"), (4, "L4")):
                self._frag(out, L[key], f"pts_linears.{i}.weight", same, False)
                self._frag(out, L[key + "T"], f"pts_linears.{i}.weight", same, True)
            for i in range(5):
                for c in range(self.nc):
                    self._frag(out, L[f"FC{i}_{c}"], f"fc_c.{i}.weight", lambda kk, c=c: 32 * c + kk, False)
                self._frag(out, L[f"FCT{i}"], f"fc_c.{i}.weight", same, True)
                self._vec(out, L["Bias"] + 32 * i, f"pts_linears.{i}.bias")
                self._vec(out, L["BiasC"] + 32 * i, f"fc_c.{i}.bias")
            offB, _ = self._w("embedder._B")
            for j in range(3):
                out[L["FB"] + 96 * j:L["FB"] + 96 * j + EMB] = offB + j * EMB + np.arange(EMB)
        else:
            for i, key in ((0, "L0"), (1, "L1"), (2, "L2"), (4, "L4")):
                self._frag(out, L[key], f"pts_linears.{i}.weight", same, False)
                self._frag(out, L[key + "T"], f"pts_linears.{i}.weight", same, True)
            for b in range(2):
                cm = lambda kk, b=b: 32 * b + kk  # noqa: E731
                self._frag(out, L["L3"] + b, "pts_linears.3.weight", cm, False)
                self._frag(out, L["L3T"] + b, "pts_linears.3.weight", cm, True)
            for i in range(5):
                self._vec(out, L["Bias"] + 32 * i, f"pts_linears.{i}.bias")
        offW, (O, K) = self._w("output_linear.weight")
        for j in range(O):
            out[L["Wo"] + 32 * j:L["Wo"] + 32 * j + K] = offW + j * K + np.arange(K)
        self._vec(out, L["Bo"], "output_linear.bias")
        return out

    # -- runtime ------------------------------------------------------------------------------
    def device_index(self, device):
        key = str(device)
        if key not in self._dev_index:
            idx = np.where(self.index >= 0, self.index, self.n_params)  # -1 → the zero slot
            self._dev_index[key] = torch.from_numpy(idx).to(device)
        return self._dev_index[key]

    def flat(self, params):
        return torch.cat([p.detach().reshape(-1) for p in params])

    def pack(self, params):
        """params in named_parameters order → packed float32 device buffer (one gather)."""
        flat = self.flat(params)
        flat = torch.cat([flat, flat.new_zeros(1)])
        return flat[self.device_index(flat.device)]

    def grad_struct(self, base: torch.Tensor | None) -> _lib.NslamDecGrad:
        g = _lib.NslamDecGrad()
        if base is None:
            return g
        g.base = base.data_ptr()
        g.count = self.n_params
        o = self.offsets
        for i in range(5):
            g.w[i] = o[f"pts_linears.{i}.weight"]
            g.b[i] = o[f"pts_linears.{i}.bias"]
            if self.kind == 0:
                g.wc[i] = o[f"fc_c.{i}.weight"]
                g.bc[i] = o[f"fc_c.{i}.bias"]
        g.wo = o["output_linear.weight"]
        g.bo = o["output_linear.bias"]
        if self.kind == 0:
            g.B = o["embedder._B"]
        return g

    def split_grad(self, flat_grad):
        """flat gradient buffer → per-parameter views (named_parameters order)."""
        return [flat_grad[self.offsets[n]:self.offsets[n] + int(np.prod(self.shapes[n]))].view(self.shapes[n])
                for n in self.names]
