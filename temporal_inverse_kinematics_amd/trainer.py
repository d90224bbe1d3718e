"""The training step on the GPU (optimizer half).

`GpuTrainer` runs what Lightning does with `IKPoseTrainer` for one batch
(pose_trainer.py:146-155 `training_step`, the backward, and the Adam step
from `configure_optimizers`, :196-197) as one stream-ordered call into
libtik.so (`tik_trainer_step`, csrc/trainer.cpp):

  * train-mode forward: BatchNorm on batch statistics with the running-stat
    momentum update (st_gcn_aaai18.py:74-75,178,186,203), Dropout(0.7) in the
    head (pose_trainer.py:91), the learnable edge importance (:104-108,129);
  * nn.MSELoss(poses, batch["poses"]) (PoseLosses, pose_trainer.py:42-50);
  * the backward of every operation and torch.optim.Adam(lr=hparams.lr).

Parameters, gradients, Adam state and BatchNorm buffers stay on the device
between steps; `state_dict()` / `load_into(module)` export them under the
reference's names (the weight ABI of SURVEY.md §8b), so a trained model
drops straight into `PoseRegressor` inference or a `.ckpt`.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from .models import IKPoseTrainer, PoseRegressor, _Handle, _state_numpy

_WHAT = {"value": 0, "grad": 1, "exp_avg": 2, "exp_avg_sq": 3}


class GpuTrainer:
    """IKPoseTrainer's training loop body on the GPU.

    >>> tr = GpuTrainer(IKPoseTrainer(hparams))      # lr = hparams.lr
    >>> out = tr.training_step(batch, 0)             # forward + MSE + backward + Adam
    >>> out["loss"], out["log"]["train/pose_mse"]
    """

    def __init__(self, model, lr: Optional[float] = None, device="cuda"):
        reg = model.regressor if isinstance(model, IKPoseTrainer) else model
        if not isinstance(reg, PoseRegressor):
            raise TypeError("GpuTrainer expects an IKPoseTrainer or PoseRegressor")
        hp = getattr(model, "hparams", None)
        if lr is None:
            lr = float(getattr(hp, "lr", 1e-4)) if hp is not None else 1e-4
        self.lr = float(lr)
        self.device = torch.device(device)
        self.regressor = reg
        named = _state_numpy(reg)
        named.append(("tik.strides", np.array(reg.backbone.strides, dtype=np.float32)))
        arr, keep = _lib.pack_tensors(named)
        lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(lib.tik_trainer_create(arr, len(named), ctypes.c_float(self.lr), ctypes.byref(h)), "GpuTrainer")
        self._h = _Handle(h.value, lib.tik_trainer_destroy)
        self._names = []
        for i in range(_lib.check(lib.tik_trainer_count(self._h.h))):
            name = ctypes.create_string_buffer(256)
            shape = (ctypes.c_int64 * 4)()
            nd, kind = ctypes.c_int(), ctypes.c_int()
            _lib.check(lib.tik_trainer_tensor(self._h.h, i, name, 256, shape, ctypes.byref(nd), ctypes.byref(kind)))
            self._names.append((name.value.decode(), tuple(shape[:nd.value]), kind.value))
        self._index = {n: i for i, (n, _, _) in enumerate(self._names)}
        self._loss = torch.zeros(1, device=self.device)
        # the BatchNorm step counters the model arrived with (checkpoint / earlier training)
        self._nbt0 = {k: int(v.item()) for k, v in reg.state_dict().items() if k.endswith("num_batches_tracked")}

    # ------------------------------------------------------------------ step
    def step(self, keypoints_3d: torch.Tensor, poses: torch.Tensor, dropout_mask: Optional[torch.Tensor] = None,
             seed: int = 0) -> torch.Tensor:
        """One optimizer step on (keypoints_3d (N,T,17,3), poses (N,T',66)); returns the
        pre-update loss as a device scalar. `dropout_mask` (N*T', 512) of 0/1 fixes the
        head's dropout draw (tests); otherwise a counter-based mask keyed by `seed`."""
        x = keypoints_3d.contiguous()
        y = poses.contiguous()
        _lib.require_gpu(x, y)
        if x.dim() != 4 or x.shape[2:] != (17, 3):
            raise ValueError(f"expected (N,T,17,3) keypoints, got {tuple(x.shape)}")
        N, T = x.shape[:2]
        lib = _lib.load()
        To = _lib.check(lib.tik_trainer_out_frames(self._h.h, T))
        if tuple(y.shape) != (N, To, self.regressor.pose_dim):
            raise ValueError(f"expected target poses {(N, To, self.regressor.pose_dim)}, got {tuple(y.shape)}")
        if x.dtype != torch.float32 or y.dtype != torch.float32:
            raise TypeError("keypoints and poses must be float32")
        mptr = None
        if dropout_mask is not None:
            dropout_mask = dropout_mask.to(self.device, torch.float32).contiguous()
            if dropout_mask.numel() != N * To * 512:
                raise ValueError("dropout_mask must hold N*T'*512 values")
            mptr = dropout_mask.data_ptr()
        _lib.check(lib.tik_trainer_step(self._h.h, x.data_ptr(), N, T, y.data_ptr(), mptr, int(seed) & (2**64 - 1),
                                        self._loss.data_ptr(), _lib.stream_of(x)), "GpuTrainer.step")
        # a fresh tensor per step (the reference returns a new loss each step;
        # the persistent device buffer is overwritten by the next step)
        return self._loss[0].clone()

    def training_step(self, batch: Dict[str, torch.Tensor], batch_idx: int = 0, dropout_mask=None):
        """pose_trainer.py:146-155 plus Lightning's backward and optimizer step."""
        loss = self.step(batch["keypoints_3d"].to(self.device), batch["poses"].to(self.device), dropout_mask,
                         seed=self.steps * 1000003 + batch_idx)
        return {"loss": loss, "log": {"train/pose_mse": loss}}

    # ------------------------------------------------------------------ state
    @property
    def steps(self) -> int:
        return int(_lib.load().tik_trainer_steps(self._h.h))

    def tensor(self, name: str, what: str = "value") -> torch.Tensor:
        i = self._index[name]
        _, shape, _ = self._names[i]
        out = torch.empty(shape, device=self.device, dtype=torch.float32)
        _lib.check(_lib.load().tik_trainer_read(self._h.h, i, _WHAT[what], out.data_ptr(),
                                                _lib.stream_of(out)), name)
        return out

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """PoseRegressor state dict after the last step (reference key names)."""
        sd = {n: self.tensor(n) for n, _, _ in self._names}
        # each BatchNorm counts on from the value it was loaded with (nn.BatchNorm increments its own buffer)
        for k, v0 in self._nbt0.items():
            sd[k] = torch.tensor(v0 + self.steps, dtype=torch.long)
        return sd

    def grads(self) -> Dict[str, torch.Tensor]:
        return {n: self.tensor(n, "grad") for n, _, k in self._names if k == 0}

    _SAVED = {"O": 0, "U": 2, "H": 3, "Z": 4, "Y": 5, "P": 6}

    def saved(self, kind: str, layer: int, shape) -> torch.Tensor:
        """The last step's saved forward activation (test / debug hook): block `layer`'s
        output "O", tcn conv output "U", post-ReLU tcn input "H", graph-mix output "Z",
        gcn conv output "Y" (channels-last (N,T,17,C)); "P" the head's first Linear
        output (N*T', 512)."""
        out = torch.empty(shape, device=self.device, dtype=torch.float32)
        _lib.check(_lib.load().tik_trainer_debug(self._h.h, self._SAVED[kind], layer, out.data_ptr(), out.numel(),
                                                 _lib.stream_of(out)), "saved")
        return out

    def load_into(self, module=None):
        """Copy the trained state into `module` (default: the regressor it was built from)."""
        reg = self.regressor if module is None else (module.regressor if isinstance(module, IKPoseTrainer) else module)
        own = reg.state_dict()
        sd = {k: v.to(own[k].device, own[k].dtype) for k, v in self.state_dict().items() if k in own}
        reg.load_state_dict(sd, strict=False)
        return reg
