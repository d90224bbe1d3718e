"""IK model modules — drop-in for `mmskeleton.models.backbones.st_gcn_aaai18`
(`StgLayerConfig`, `StgConfig`, `StgGcn18`, `StGcnBlock`) and the model half of
`pose_trainer.py` (`PoseRegressor`, `IKPoseTrainer`).

The modules keep the reference's parameter/buffer names, so a reference state
dict (or the `regressor.*` part of its Lightning checkpoint) loads unchanged.
The torch parameters are only storage: `forward` hands them, once per weight
version, to libtik.so (BN folded and packed on the host, uploaded once) and
runs the fused HIP path. Eval semantics only (BatchNorm running stats,
Dropout identity) — the path the reference's `inference.py` uses.
"""
from __future__ import annotations

import argparse
from dataclasses import dataclass
from typing import List

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .st_gcn import ConvTemporalGraphical, Graph


def zero(x):
    return 0


def iden(x):
    return x


@dataclass
class StgLayerConfig:
    """st_gcn_aaai18.py:18-23"""
    in_channels: int
    out_channels: int
    temporal_stride: int
    is_residual: True


@dataclass
class StgConfig:
    """st_gcn_aaai18.py:26-29"""
    layers: List[StgLayerConfig]
    temporal_kernel_size: int


def _create_model_handle(named):
    lib = _lib.load()
    arr, keep = _lib.pack_tensors(named)
    h = _lib.ctypes.c_void_p()
    _lib.check(lib.tik_model_create(arr, len(named), _lib.ctypes.byref(h)), "tik_model_create")
    return _Handle(h.value, lib.tik_model_destroy)


def _state_numpy(module: nn.Module, prefix: str = ""):
    out = []
    for k, v in module.state_dict(prefix=prefix).items():
        if k.endswith("num_batches_tracked"):
            continue
        out.append((k, v.detach().to("cpu", torch.float32).numpy()))
    return out


def _weights_key(module: nn.Module):
    return tuple((t.data_ptr(), t._version) for t in list(module.parameters()) + list(module.buffers()))


class _Handle:
    """Owns a libtik handle; destroyed with the module."""

    def __init__(self, h, destroy):
        self.h = h
        self._destroy = destroy

    def __del__(self):
        try:
            if self.h:
                self._destroy(self.h)
        except Exception:
            pass


class StGcnBlock(nn.Module):
    """st_gcn_aaai18.py:136-214. forward(x (N,Cin,T,V), A (1,V,V)) -> (x', A)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, dropout=0, residual=True):
        super().__init__()
        assert len(kernel_size) == 2
        assert kernel_size[0] % 2 == 1
        padding = ((kernel_size[0] - 1) // 2, 0)
        self.in_channels, self.out_channels, self.stride = in_channels, out_channels, stride
        self.has_residual = bool(residual)
        self.gcn = ConvTemporalGraphical(in_channels, out_channels, kernel_size[1])
        self.tcn = nn.Sequential(
            nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
            nn.Conv2d(out_channels, out_channels, (kernel_size[0], 1), (stride, 1), padding),
            nn.BatchNorm2d(out_channels),
            nn.Dropout(dropout, inplace=True),
        )
        if not residual:
            self.residual = zero
        elif in_channels == out_channels and stride == 1:
            self.residual = iden
        else:
            self.residual = nn.Sequential(
                nn.Conv2d(in_channels, out_channels, kernel_size=1, stride=(stride, 1)),
                nn.BatchNorm2d(out_channels),
            )
        self.relu = nn.ReLU(inplace=True)
        self._tik = None
        self._tik_key = None
        self.tik_precision = None

    def _handle(self, A: torch.Tensor):
        if self.training:
            raise NotImplementedError("the HIP path implements eval-mode StGcnBlock only; call .eval()")
        if A.dim() != 3 or A.shape[0] != 1:
            raise ValueError("the fused block kernel supports the 'uniform' strategy (K=1) only")
        a_host = A[0].detach().to("cpu", torch.float32).contiguous().numpy()
        key = (_weights_key(self), a_host.tobytes())
        if self._tik is None or self._tik_key != key:
            lib = _lib.load()
            arr, keep = _lib.pack_tensors(_state_numpy(self))
            h = _lib.ctypes.c_void_p()
            V = a_host.shape[0]
            _lib.check(lib.tik_block_create(arr, len(keep) // 2, self.in_channels, self.out_channels, self.stride,
                                            int(self.has_residual),
                                            a_host.ctypes.data_as(_lib._F), V, _lib.ctypes.byref(h)),
                       "StGcnBlock")
            self._tik = _Handle(h.value, lib.tik_block_destroy)
            self._tik_key = key
        if self.tik_precision is not None:
            _lib.check(_lib.load().tik_block_set_precision(self._tik.h, _lib.precision_code(self.tik_precision)))
        return self._tik.h

    def forward(self, x, A):
        h = self._handle(A)
        _lib.require_gpu(x.contiguous())
        N, C, T, V = x.shape
        if C != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {C}")
        xl = x.permute(0, 2, 3, 1).contiguous()                       # channels-last (N,T,V,C)
        To = (T - 1) // self.stride + 1
        out = torch.empty((N, To, V, self.out_channels), device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().tik_stgcn_block_fwd(h, xl.data_ptr(), N, T, out.data_ptr(), _lib.stream_of(x)),
                   "StGcnBlock")
        return out.permute(0, 3, 1, 2).contiguous(), A


class StgGcn18(nn.Module):
    """st_gcn_aaai18.py:32-133. forward(x (N,T,V,C)) -> (N,T',V*Cout)."""

    def __init__(self, config: StgConfig, graph_cfg, edge_importance_weighting=True, data_bn=True, **kwargs):
        super().__init__()
        self.graph = Graph(**graph_cfg)
        A = torch.tensor(self.graph.A, dtype=torch.float32, requires_grad=False)
        self.register_buffer("A", A)
        self.n_in_keypoints = A.size(1)
        spatial_kernel_size = A.size(0)
        kernel_size = (config.temporal_kernel_size, spatial_kernel_size)
        in_channels = config.layers[0].in_channels
        if not data_bn:
            raise ValueError("the fused path folds data_bn; data_bn=False is not supported")
        self.data_bn = nn.BatchNorm1d(in_channels * A.size(1))
        kwargs0 = {k: v for k, v in kwargs.items() if k != "dropout"}
        self.st_gcn_networks = nn.ModuleList([
            StGcnBlock(layer.in_channels, layer.out_channels, kernel_size, stride=layer.temporal_stride,
                       residual=layer.is_residual, **kwargs0)
            for layer in config.layers])
        if not edge_importance_weighting:
            raise ValueError("edge_importance_weighting=False is not supported by the fused path")
        self.edge_importance = nn.ParameterList([nn.Parameter(torch.ones(self.A.size()))
                                                 for _ in self.st_gcn_networks])
        self.strides = [layer.temporal_stride for layer in config.layers]
        self.out_channels = config.layers[-1].out_channels
        self._tik = None
        self._tik_key = None
        self.tik_precision = None   # None: library default (bf16x3); "fp32" | "bf16x3"

    def out_frames(self, T: int) -> int:
        for s in self.strides:
            T = (T - 1) // s + 1
        return T

    def tik_handle(self):
        """A backbone-only libtik handle for the current weights (rebuilt when they change)."""
        if self.training:
            raise NotImplementedError("the HIP path implements eval-mode inference only; call .eval()")
        key = _weights_key(self)
        if self._tik is None or self._tik_key != key:
            named = _state_numpy(self, prefix="backbone.")
            named.append(("tik.strides", np.array(self.strides, dtype=np.float32)))
            self._tik = _create_model_handle(named)
            self._tik_key = key
        if self.tik_precision is not None:
            _lib.check(_lib.load().tik_model_set_precision(self._tik.h, _lib.precision_code(self.tik_precision)))
        return self._tik.h

    def forward(self, x):
        """st_gcn_aaai18.py:113-133: x (N,T,V,C) -> (N,T',V*Cout), feature index
        v*Cout + c (data_bn, the 8 blocks with A * edge_importance, flatten) —
        one tik_backbone_forward call."""
        if x.dim() != 4:
            raise ValueError(f"expected (N,T,V,C) keypoints, got shape {tuple(x.shape)}")
        N, T, V, C = x.shape
        To = self.out_frames(T)
        if N == 0:
            return torch.empty((0, To, V * self.out_channels), device=x.device, dtype=torch.float32)
        x = x.contiguous()
        _lib.require_gpu(x)
        h = self.tik_handle()
        feat = torch.empty((N, To, V * self.out_channels), device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().tik_backbone_forward(h, x.data_ptr(), N, T, feat.data_ptr(), _lib.stream_of(x)),
                   "StgGcn18")
        return feat


class PoseRegressor(nn.Module):
    """pose_trainer.py:66-133: StgGcn18 (8-layer config) + MLP head -> {'poses': (N,T',66)}."""

    LAYERS = [(64, 1), (64, 1), (128, 2), (128, 1), (128, 1), (128, 2), (256, 2), (256, 2)]

    def __init__(self, hparams):
        super().__init__()
        self.graph_cfg = dict(layout=hparams.graph_layout, strategy="uniform", max_hop=hparams.max_hop,
                              dilation=hparams.dilation)
        c = hparams.kps_channel
        layers = []
        for cout, s in self.LAYERS:
            layers.append(StgLayerConfig(in_channels=c, out_channels=cout, temporal_stride=s, is_residual=True))
            c = cout
        self.backbone = StgGcn18(config=StgConfig(layers=layers, temporal_kernel_size=3), graph_cfg=self.graph_cfg)
        self.pose_dim = 22 * 3
        self.pose_regressor = nn.Sequential(nn.Linear(17 * 256, 512), nn.LeakyReLU(), nn.Dropout(0.7),
                                            nn.Linear(512, self.pose_dim))
        self._tik = None
        self._tik_key = None
        self.tik_precision = None   # None: library default (bf16x3); "fp32" | "bf16x3"

    def tik_handle(self):
        """The libtik model handle for the current weights (rebuilt when they change)."""
        if self.training:
            raise NotImplementedError("the HIP path implements eval-mode inference only; call .eval()")
        key = _weights_key(self)
        if self._tik is None or self._tik_key != key:
            named = _state_numpy(self)
            named.append(("tik.strides", np.array(self.backbone.strides, dtype=np.float32)))
            self._tik = _create_model_handle(named)
            self._tik_key = key
        if self.tik_precision is not None:
            _lib.check(_lib.load().tik_model_set_precision(self._tik.h, _lib.precision_code(self.tik_precision)))
        return self._tik.h

    def forward(self, x, init_pose=None, n_iter=3):
        if x.dim() != 4:
            raise ValueError(f"expected (N,T,V,C) keypoints, got shape {tuple(x.shape)}")
        N, T, V, C = x.shape
        To = self.backbone.out_frames(T)
        if N == 0:   # an empty batch (e.g. an empty rank shard): empty poses, as torch would give
            return {"poses": torch.empty((0, To, self.pose_dim), device=x.device, dtype=torch.float32)}
        x = x.contiguous()
        _lib.require_gpu(x)
        h = self.tik_handle()
        poses = torch.empty((N, To, self.pose_dim), device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().tik_ik_forward(h, x.data_ptr(), N, T, poses.data_ptr(), _lib.stream_of(x)),
                   "PoseRegressor")
        return {"poses": poses}

    def backbone_features(self, x):
        """StgGcn18.forward output (N,T',17*256) through the fused path."""
        N, T = x.shape[:2]
        To = self.backbone.out_frames(T)
        if N == 0:
            return torch.empty((0, To, 17 * 256), device=x.device, dtype=torch.float32)
        h = self.tik_handle()
        x = x.contiguous()
        _lib.require_gpu(x)
        feat = torch.empty((N, To, 17 * 256), device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().tik_backbone_forward(h, x.data_ptr(), N, T, feat.data_ptr(), _lib.stream_of(x)),
                   "StgGcn18")
        return feat


def default_hparams(win_size: int = 9) -> argparse.Namespace:
    """The argparse defaults of IKPoseTrainer.add_model_specific_args (pose_trainer.py:204-230)."""
    return argparse.Namespace(lr=1e-4, win_size=win_size, bs=256, kps_channel=3, graph_layout="coco",
                              max_hop=2, dilation=1, keypoint_format="coco", n_out_joints=22, n_out_channels=3)


class IKPoseTrainer(nn.Module):
    """The model wrapper `inference.py` drives (pose_trainer.py:135-144):
    `.hparams` (win_size), `.regressor`, `.device`, forward -> regressor(x).
    Lightning training hooks are out of scope."""

    def __init__(self, hparams):
        super().__init__()
        self.hparams = hparams
        self.regressor = PoseRegressor(hparams)

    @property
    def device(self):
        return next(self.parameters()).device

    def forward(self, keypoints_3d):
        return self.regressor(keypoints_3d)

    @classmethod
    def load_from_checkpoint(cls, path, hparams=None, map_location="cpu"):
        """Lightning `.ckpt` reader (pose_trainer.py:240-256, inference.py:136): the
        `state_dict` entries (keys `regressor.*`) and `hparams`. Loaded with
        torch.load(weights_only=True); argparse.Namespace is allow-listed."""
        torch.serialization.add_safe_globals([argparse.Namespace])
        ck = torch.load(path, map_location=map_location, weights_only=True)
        hp = hparams
        if hp is None:
            h = ck.get("hparams", ck.get("hyper_parameters"))
            if isinstance(h, dict):
                base = vars(default_hparams())
                base.update(h)
                h = argparse.Namespace(**base)
            hp = h if h is not None else default_hparams()
        model = cls(hp)
        sd = ck["state_dict"] if "state_dict" in ck else ck
        model.load_checked_state_dict(sd)
        return model

    def load_checked_state_dict(self, sd):
        """load_state_dict that fails loudly on any key mismatch. The only keys
        allowed to be absent are BatchNorm `num_batches_tracked` counters
        (checkpoints from torch versions before they existed); eval never reads
        them. A `regressor.` prefix is required, as in the reference's Lightning
        checkpoints (IKPoseTrainer.regressor, pose_trainer.py:139)."""
        res = self.load_state_dict(sd, strict=False)
        missing = [k for k in res.missing_keys if not k.endswith("num_batches_tracked")]
        if missing or res.unexpected_keys:
            raise KeyError(f"checkpoint does not match IKPoseTrainer: missing {missing[:8]}"
                           f"{'...' if len(missing) > 8 else ''} ({len(missing)}), unexpected "
                           f"{list(res.unexpected_keys)[:8]} ({len(res.unexpected_keys)})")
        return res
