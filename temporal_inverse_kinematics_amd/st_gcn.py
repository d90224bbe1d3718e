"""Graph-convolution operator API — drop-in for `mmskeleton.ops.st_gcn`
(`mmskeleton/ops/st_gcn/__init__.py:1-2`): `ConvTemporalGraphical`, `Graph`.

`Graph` is host-side constant construction (numpy, float64, as the reference).
`ConvTemporalGraphical.forward` runs the HIP kernel `tik_gconv_fwd` on the GPU;
there is no CPU path.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _lib

_LAYOUTS = {
    # layout: (num_node, 0-based neighbour links, center)   graph.py:38-85
    "openpose": (18, [(4, 3), (3, 2), (7, 6), (6, 5), (13, 12), (12, 11), (10, 9), (9, 8),
                      (11, 5), (8, 2), (5, 1), (2, 1), (0, 1), (15, 0), (14, 0), (17, 15),
                      (16, 14)], 1),
    "ntu-rgb+d": (25, [(a - 1, b - 1) for a, b in [
        (1, 2), (2, 21), (3, 21), (4, 3), (5, 21), (6, 5), (7, 6), (8, 7), (9, 21), (10, 9),
        (11, 10), (12, 11), (13, 1), (14, 13), (15, 14), (16, 15), (17, 1), (18, 17), (19, 18),
        (20, 19), (22, 23), (23, 8), (24, 25), (25, 12)]], 20),
    "ntu_edge": (24, [(a - 1, b - 1) for a, b in [
        (1, 2), (3, 2), (4, 3), (5, 2), (6, 5), (7, 6), (8, 7), (9, 2), (10, 9), (11, 10),
        (12, 11), (13, 1), (14, 13), (15, 14), (16, 15), (17, 1), (18, 17), (19, 18), (20, 19),
        (21, 22), (22, 8), (23, 24), (24, 12)]], 2),
    "coco": (17, [(a - 1, b - 1) for a, b in [
        (16, 14), (14, 12), (17, 15), (15, 13), (12, 13), (6, 12), (7, 13), (6, 7), (8, 6),
        (9, 7), (10, 8), (11, 9), (2, 3), (2, 1), (3, 1), (4, 2), (5, 3), (4, 6), (5, 7)]], 0),
}


def get_hop_distance(num_node, edge, max_hop=1):
    """Hop distance (inf when unreachable) — graph.py:136-148."""
    adj = np.zeros((num_node, num_node))
    for i, j in edge:
        adj[j, i] = adj[i, j] = 1
    hop = np.full((num_node, num_node), np.inf)
    reach = np.stack([np.linalg.matrix_power(adj, d) for d in range(max_hop + 1)]) > 0
    for d in range(max_hop, -1, -1):
        hop[reach[d]] = d
    return hop


def normalize_digraph(A):
    """A @ diag(1/colsum) (zero columns stay zero) — graph.py:151-159."""
    col = A.sum(0)
    inv = np.zeros_like(col)
    nz = col > 0
    inv[nz] = 1.0 / col[nz]
    return A @ np.diag(inv)


def normalize_undigraph(A):
    """D^-1/2 A D^-1/2 — graph.py:162-170."""
    col = A.sum(0)
    inv = np.zeros_like(col)
    nz = col > 0
    inv[nz] = col[nz] ** -0.5
    d = np.diag(inv)
    return d @ A @ d


class Graph:
    """Skeleton graph and its (K, V, V) adjacency — graph.py:4-133.

    Same constructor, attributes (`A`, `num_node`, `edge`, `center`, `hop_dis`,
    `max_hop`, `dilation`) and ValueError messages as the reference.
    """

    def __init__(self, layout="openpose", strategy="uniform", max_hop=1, dilation=1):
        self.max_hop = max_hop
        self.dilation = dilation
        self.get_edge(layout)
        self.hop_dis = get_hop_distance(self.num_node, self.edge, max_hop=max_hop)
        self.get_adjacency(strategy)

    def __str__(self):
        return str(self.A)

    def get_edge(self, layout):
        if layout not in _LAYOUTS:
            raise ValueError("Do Not Exist This Layout.")
        n, links, center = _LAYOUTS[layout]
        self.num_node = n
        self.edge = [(i, i) for i in range(n)] + list(links)
        self.center = center

    def get_adjacency(self, strategy):
        valid_hop = range(0, self.max_hop + 1, self.dilation)
        n = self.num_node
        adjacency = np.zeros((n, n))
        for hop in valid_hop:
            adjacency[self.hop_dis == hop] = 1
        norm = normalize_digraph(adjacency)
        if strategy == "uniform":
            self.A = norm[None].copy()
        elif strategy == "distance":
            A = np.zeros((len(valid_hop), n, n))
            for i, hop in enumerate(valid_hop):
                m = self.hop_dis == hop
                A[i][m] = norm[m]
            self.A = A
        elif strategy == "spatial":
            hc = self.hop_dis[:, self.center]           # hop of each node to the center
            parts = []
            for hop in valid_hop:
                on = self.hop_dis == hop                   # [j, i]
                closer = hc[:, None] > hc[None, :]         # hop(j,c) > hop(i,c)
                same = hc[:, None] == hc[None, :]
                root = np.where(on & same, norm, 0.0)
                close = np.where(on & closer, norm, 0.0)
                far = np.where(on & ~same & ~closer, norm, 0.0)
                if hop == 0:
                    parts.append(root)
                else:
                    parts.append(root + close)
                    parts.append(far)
            self.A = np.stack(parts)
        else:
            raise ValueError("Do Not Exist This Strategy")


class ConvTemporalGraphical(nn.Module):
    """gconv_origin.py:8-65 — Conv2d((t_kernel,1)) to K*Cout channels, then the
    per-frame graph mix einsum('nkctv,kvw->nctw'). Runs `tik_gconv_fwd`."""

    def __init__(self, in_channels, out_channels, kernel_size, t_kernel_size=1, t_stride=1,
                 t_padding=0, t_dilation=1, bias=True):
        super().__init__()
        self.kernel_size = kernel_size
        self.conv = nn.Conv2d(in_channels, out_channels * kernel_size, kernel_size=(t_kernel_size, 1),
                              padding=(t_padding, 0), stride=(t_stride, 1), dilation=(t_dilation, 1),
                              bias=bias)

    def forward(self, x, A):
        assert A.size(0) == self.kernel_size
        lib = _lib.load()
        x = x.contiguous()
        A = A.to(device=x.device, dtype=torch.float32).contiguous()
        w = self.conv.weight.contiguous()
        b = self.conv.bias.contiguous() if self.conv.bias is not None else None
        _lib.require_gpu(x, A, w, b)
        N, Cin, T, V = x.shape
        K = self.kernel_size
        Cout = w.shape[0] // K
        tk, ts = self.conv.kernel_size[0], self.conv.stride[0]
        tp, td = self.conv.padding[0], self.conv.dilation[0]
        To = (T + 2 * tp - td * (tk - 1) - 1) // ts + 1
        if To <= 0:
            raise ValueError(f"temporal output length {To} <= 0")
        out = torch.empty((N, Cout, To, V), device=x.device, dtype=torch.float32)
        _lib.check(lib.tik_gconv_fwd(x.data_ptr(), N, Cin, T, V, A.data_ptr(), K, w.data_ptr(), _lib.ptr(b),
                                     Cout, tk, ts, tp, td, out.data_ptr(), _lib.stream_of(x)),
                   "ConvTemporalGraphical")
        return out, A
