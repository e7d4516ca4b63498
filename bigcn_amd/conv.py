"""Drop-in ``torch_geometric.nn.GCNConv`` (PyG >= 2.0 layout) on the HIP kernels.

Reference usage: ``GCNConv(in_feats, hid_feats)`` / ``GCNConv(hid_feats+in_feats, out_feats)``
at ``model/Twitter/BiGCN_Twitter.py:22-23,73-74`` (Weibo ``:19-20,49-50``), called as
``conv(x, edge_index)``.  The state_dict keys match PyG 2.x (``lin.weight [out, in]``,
``bias [out]``), so checkpoints written by the reference (``tools/earlystopping.py:59-69``)
load unchanged.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from .ops import Graph, degree_code, gcn_conv


class _Lin(torch.nn.Module):
    """``torch_geometric.nn.dense.Linear(in, out, bias=False, weight_initializer='glorot')``."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight = torch.nn.Parameter(torch.empty(out_channels, in_channels))
        self.reset_parameters()

    def reset_parameters(self):
        a = math.sqrt(6.0 / (self.weight.size(-2) + self.weight.size(-1)))  # glorot
        with torch.no_grad():
            self.weight.uniform_(-a, a)


class GCNConv(torch.nn.Module):
    """``GCNConv(in_channels, out_channels, improved=False, cached=False, add_self_loops=True,
    normalize=True, bias=True)``; ``degree_on='row'`` selects the PyG 1.3.2 convention."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = True, degree_on: str = "col"):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        degree_code(degree_on)
        self.degree_on = degree_on
        self.lin = _Lin(in_channels, out_channels)
        if bias:
            self.bias = torch.nn.Parameter(torch.zeros(out_channels))
        else:
            self.register_parameter("bias", None)

    def reset_parameters(self):
        self.lin.reset_parameters()
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x: torch.Tensor, edge_index, edge_weight: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``edge_index`` may also be a prebuilt :class:`Graph` (built once per batch)."""
        return gcn_conv(x, edge_index, self.lin.weight, self.bias, edge_weight, self.degree_on)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"
