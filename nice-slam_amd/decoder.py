"""NICE decoders with the reference's module structure and state_dict keys.

Mirrors src/conv_onet/models/decoder.py (GaussianFourierFeatureTransform :7-30, DenseLayer
:70-79, MLP :91-203, MLP_no_xyz :206-274, NICE :277-342) so checkpoints / pretrained decoders
load unchanged (`fc_c.i`, `pts_linears.i`, `output_linear`, `embedder._B`).  The forward pass is
the fused HIP query (ops.query_points): one kernel evaluates the whole stage (grid lookups,
Fourier features, the MLPs and the stage combiner) per 32-point tile.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import ops
from .packing import DecoderPacker


class GaussianFourierFeatureTransform(nn.Module):
    """sin(x @ B), B ~ N(0,1)*scale, [3, 93], learnable (decoder.py:7-30)."""

    def __init__(self, num_input_channels, mapping_size=93, scale=25, learnable=True):
        super().__init__()
        B = torch.randn((num_input_channels, mapping_size)) * scale
        if learnable:
            self._B = nn.Parameter(B)
        else:
            self.register_buffer("_B", B, persistent=False)


class DenseLayer(nn.Linear):
    """nn.Linear with xavier-uniform(gain(activation)) weights and zero bias (decoder.py:70-79)."""

    def __init__(self, in_dim: int, out_dim: int, activation: str = "relu", *args, **kwargs) -> None:
        self.activation = activation
        super().__init__(in_dim, out_dim, *args, **kwargs)

    def reset_parameters(self) -> None:
        nn.init.xavier_uniform_(self.weight, gain=nn.init.calculate_gain(self.activation))
        if self.bias is not None:
            nn.init.zeros_(self.bias)


def _check_supported(hidden_size, n_blocks, skips, leaky, sample_mode):
    if hidden_size != 32 or n_blocks != 5 or list(skips) != [2] or leaky or sample_mode != "bilinear":
        raise NotImplementedError(
            "the fused HIP decoder implements NICE-SLAM's configuration (hidden 32, 5 blocks, skip after "
            "block 2, ReLU, bilinear sampling; configs/nice_slam.yaml)")


class MLP(nn.Module):
    """Middle / fine / color decoder (decoder.py:91-203); forward through the fused kernel."""

    def __init__(self, name="", dim=3, c_dim=128, hidden_size=256, n_blocks=5, leaky=False, sample_mode="bilinear",
                 color=False, skips=[2], grid_len=0.16, pos_embedding_method="fourier", concat_feature=False):
        super().__init__()
        _check_supported(hidden_size, n_blocks, skips, leaky, sample_mode)
        if pos_embedding_method != "fourier" or dim != 3:
            raise NotImplementedError("NICE-SLAM uses the Fourier embedding (configs/nice_slam.yaml:116)")
        expect_c = 64 if concat_feature else 32
        if c_dim != expect_c:
            raise NotImplementedError(f"c_dim must be {expect_c} for decoder {name!r} (grid channels = 32)")
        self.name = name
        self.color = color
        self.no_grad_feature = False
        self.c_dim = c_dim
        self.grid_len = grid_len
        self.concat_feature = concat_feature
        self.n_blocks = n_blocks
        self.skips = skips
        self.fc_c = nn.ModuleList([nn.Linear(c_dim, hidden_size) for _ in range(n_blocks)])
        embedding_size = 93
        self.embedder = GaussianFourierFeatureTransform(dim, mapping_size=embedding_size, scale=25)
        self.pts_linears = nn.ModuleList(
            [DenseLayer(embedding_size, hidden_size, activation="relu")]
            + [DenseLayer(hidden_size, hidden_size, activation="relu") if i not in skips
               else DenseLayer(hidden_size + embedding_size, hidden_size, activation="relu")
               for i in range(n_blocks - 1)])
        self.output_linear = DenseLayer(hidden_size, 4 if color else 1, activation="linear")
        self.sample_mode = sample_mode
        self.bound = None
        self._packer = None

    def packer(self):
        if self._packer is None:
            self._packer = DecoderPacker(self, kind=0, nc=2 if self.concat_feature else 1,
                                         nout=4 if self.color else 1)
        return self._packer

    def forward(self, p, c_grid=None):
        """decoder.py:177-203 for this decoder alone (NICE.forward evaluates a whole stage in one
        fused launch instead): occupancy [P] (middle, fine) or [P, 4] (colour).

        Colour decoder: all four output columns are differentiable, as in the reference module —
        the 4th (which NICE.forward overwrites with the occupancy, decoder.py:341) reaches
        output_linear's row 3 through torch and the hidden layers, grid and points through the
        kernels' h4 cotangent (ABI v17 nslam_query_cfg.g_h4; tests/test_gpu_decoders.py)."""
        return ops.query_decoder(self, p, c_grid)


class MLP_no_xyz(nn.Module):
    """Coarse decoder (decoder.py:206-274)."""

    def __init__(self, name="", dim=3, c_dim=128, hidden_size=256, n_blocks=5, leaky=False, sample_mode="bilinear",
                 color=False, skips=[2], grid_len=0.16):
        super().__init__()
        _check_supported(hidden_size, n_blocks, skips, leaky, sample_mode)
        if c_dim != 32 or color:
            raise NotImplementedError("the coarse decoder reads a 32-channel grid and outputs occupancy")
        self.name = name
        self.no_grad_feature = False
        self.color = color
        self.grid_len = grid_len
        self.c_dim = c_dim
        self.n_blocks = n_blocks
        self.skips = skips
        self.pts_linears = nn.ModuleList(
            [DenseLayer(hidden_size, hidden_size, activation="relu")]
            + [DenseLayer(hidden_size, hidden_size, activation="relu") if i not in skips
               else DenseLayer(hidden_size + c_dim, hidden_size, activation="relu") for i in range(n_blocks - 1)])
        self.output_linear = DenseLayer(hidden_size, 1, activation="linear")
        self.sample_mode = sample_mode
        self.bound = None
        self._packer = None

    def packer(self):
        if self._packer is None:
            self._packer = DecoderPacker(self, kind=1)
        return self._packer

    def forward(self, p, c_grid, **kwargs):
        """decoder.py:262-274: coarse occupancy [P] (the grid is read over the enlarged bound)."""
        return ops.query_decoder(self, p, c_grid)


class NICE(nn.Module):
    """Hierarchical decoder (decoder.py:277-342).  forward(p[1,P,3] or [P,3], c_grid, stage) → raw [P,4]."""

    def __init__(self, dim=3, c_dim=32, coarse_grid_len=2.0, middle_grid_len=0.16, fine_grid_len=0.16,
                 color_grid_len=0.16, hidden_size=32, coarse=False, pos_embedding_method="fourier"):
        super().__init__()
        if coarse:
            self.coarse_decoder = MLP_no_xyz(name="coarse", dim=dim, c_dim=c_dim, color=False,
                                             hidden_size=hidden_size, grid_len=coarse_grid_len)
        self.middle_decoder = MLP(name="middle", dim=dim, c_dim=c_dim, color=False, skips=[2], n_blocks=5,
                                  hidden_size=hidden_size, grid_len=middle_grid_len,
                                  pos_embedding_method=pos_embedding_method)
        self.fine_decoder = MLP(name="fine", dim=dim, c_dim=c_dim * 2, color=False, skips=[2], n_blocks=5,
                                hidden_size=hidden_size, grid_len=fine_grid_len, concat_feature=True,
                                pos_embedding_method=pos_embedding_method)
        self.color_decoder = MLP(name="color", dim=dim, c_dim=c_dim, color=True, skips=[2], n_blocks=5,
                                 hidden_size=hidden_size, grid_len=color_grid_len,
                                 pos_embedding_method=pos_embedding_method)
        self.bound = None

    def decoder(self, name):
        return getattr(self, name + "_decoder")

    def set_bound(self, bound, coarse_bound_enlarge=2.0):
        """What NICE_SLAM.load_bound does to the decoders (src/NICE_SLAM.py:151-157)."""
        self.bound = bound
        self.middle_decoder.bound = bound
        self.fine_decoder.bound = bound
        self.color_decoder.bound = bound
        if hasattr(self, "coarse_decoder"):
            self.coarse_decoder.bound = bound * coarse_bound_enlarge

    def forward(self, p, c_grid, stage="middle", oob_bound=None, **kwargs):
        return ops.query_points(self, p.reshape(-1, 3), c_grid, stage, oob_bound=oob_bound)


def xavier_bound(fan_in, fan_out, gain):
    return gain * math.sqrt(6.0 / (fan_in + fan_out))
