"""Online (streaming) IK — BASELINE.json config #5.

The reference is offline: `inference.run_inference` (inference.py:37-67)
solves a recorded sequence with one edge-padded window per frame. Online,
frame c is solvable once frame c+h has arrived (h = win_size//2); each
`push` appends a frame to a device ring, gathers the window centred h frames
back and solves it (`tik_stream_*`). Output for frame c is identical to
run_inference's (within fp32 rounding). The default step is one dataflow
kernel (csrc/online.hip) over only the frames pose row 0 depends on, its convs
in bf16x3 MFMA arithmetic (`path == "dataflow"`); TIK_ONLINE=0 selects the
layered forward over the whole window.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import _lib


class OnlineIK:
    def __init__(self, model, win_size: Optional[int] = None, use_graph: bool = True):
        reg = getattr(model, "regressor", model)
        self.win_size = int(win_size if win_size is not None else model.hparams.win_size)
        self.h = self.win_size // 2
        self._model = model
        lib = _lib.load()
        handle = reg.tik_handle()
        # the stream owns its workspace and holds a library reference on the
        # model handle, so later batch calls (which may grow the handle's
        # workspace) or a handle rebuilt after a weight change leave it intact;
        # the Python reference below only documents that ownership
        self._handle_ref = reg._tik
        s = _lib.ctypes.c_void_p()
        _lib.check(lib.tik_stream_create(handle, self.win_size, int(use_graph), _lib.ctypes.byref(s)), "OnlineIK")
        self._s = s.value
        self._destroy = lib.tik_stream_destroy
        self._pose = np.zeros(66, np.float32)
        self._last = None
        # per-push overhead: the frame goes through one preallocated buffer and both
        # ctypes pointers are made once (building them per call cost ~8 us of a ~60 us push)
        self._push_fn = lib.tik_stream_push
        self._fbuf = np.zeros(51, np.float32)
        self._fptr = self._fbuf.ctypes.data_as(_lib._F)
        self._pptr = self._pose.ctypes.data_as(_lib._F)
        self.path = "dataflow" if _lib.check(lib.tik_stream_path(self._s)) == 1 else "layered"

    def __del__(self):
        try:
            if getattr(self, "_s", None):
                self._destroy(self._s)
        except Exception:
            pass

    def reset(self):
        _lib.check(_lib.load().tik_stream_reset(self._s))
        self._last = None

    def push(self, frame: np.ndarray) -> Optional[np.ndarray]:
        """frame (17,3) -> the (66,) pose of the frame h pushes back, or None while filling."""
        f = np.asarray(frame, dtype=np.float32)
        if f.size != 51:
            raise ValueError("expected one (17,3) COCO frame")
        self._fbuf[:] = f.reshape(-1)
        self._last = self._fbuf   # the last pushed frame (flush repeats it)
        rc = self._push_fn(self._s, self._fptr, self._pptr)
        if rc < 0:
            _lib.check(rc, "OnlineIK.push")
        return self._pose.copy() if rc == 1 else None

    def flush(self):
        """Poses of the last h frames (right edge padding = repeat the last frame)."""
        out = []
        for _ in range(self.h):
            p = self.push(self._last.reshape(17, 3))
            if p is not None:
                out.append(p)
        return out

    def run(self, seq: np.ndarray) -> np.ndarray:
        """Whole sequence through the online path: (F,17,3) -> (F,66)."""
        self.reset()
        out = []
        for fr in seq:
            p = self.push(fr)
            if p is not None:
                out.append(p)
        out += self.flush()
        return np.stack(out)[: seq.shape[0]]
