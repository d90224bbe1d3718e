"""CPU-side checks: the C-ABI library loads and exports every symbol of
include/tik.h (no compute calls), and the host-side mirror of the reference
interface (Graph, windowing, keypoint maps, synthetic data) matches the
reference's golden vectors."""
import os
import re

import numpy as np
import pytest

from conftest import REPO, golden


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "tik.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(tik_\w+)\s*\(", txt, re.M)))


def test_library_exports_header_symbols():
    from temporal_inverse_kinematics_amd import _build, _lib
    _build.build()
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), f"libtik.so does not export {s}"
        assert s in _lib.SIGNATURES, f"_lib.SIGNATURES lacks {s}"
    assert b"gfx950" in lib.tik_version()


def test_library_rejects_bad_args_without_gpu():
    from temporal_inverse_kinematics_amd import _lib
    lib = _lib.load()
    with pytest.raises(ValueError):
        _lib.check(lib.tik_ik_forward(None, None, 0, 0, None, None))
    assert "bad arguments" in _lib.last_error()
    arr, keep = _lib.pack_tensors([("foo", np.zeros(3, np.float32))])
    h = _lib.ctypes.c_void_p()
    with pytest.raises(KeyError):
        _lib.check(lib.tik_model_create(arr, 1, _lib.ctypes.byref(h)))


def test_trainer_abi_rejects_bad_args_without_gpu():
    """The training-step C ABI validates before touching the device: a state dict
    without the layer strides is a KeyError, null handles / bad reads ValueError."""
    from temporal_inverse_kinematics_amd import _lib
    lib = _lib.load()
    arr, keep = _lib.pack_tensors([("backbone.data_bn.weight", np.ones(51, np.float32))])
    h = _lib.ctypes.c_void_p()
    with pytest.raises(KeyError, match="tik.strides"):
        _lib.check(lib.tik_trainer_create(arr, 1, _lib.ctypes.c_float(1e-4), _lib.ctypes.byref(h)))
    with pytest.raises(ValueError):
        _lib.check(lib.tik_trainer_create(arr, 1, _lib.ctypes.c_float(0.0), _lib.ctypes.byref(h)))
    with pytest.raises(ValueError):
        _lib.check(lib.tik_trainer_step(None, None, 1, 9, None, None, 0, None, None))
    with pytest.raises(ValueError):
        _lib.check(lib.tik_trainer_read(None, 0, 0, None, None))
    assert lib.tik_trainer_steps(None) == -1


def test_graph_matches_reference():
    from temporal_inverse_kinematics_amd.st_gcn import Graph
    g = golden("graph.npz")
    for key in g.files:
        layout, strategy, hop = key.split("|")[:3]
        G = Graph(layout, strategy, int(hop), 1)
        if key.endswith("|hop"):
            np.testing.assert_array_equal(np.where(np.isinf(G.hop_dis), -1, G.hop_dis), g[key])
        else:
            np.testing.assert_allclose(G.A, g[key], atol=1e-15)
    with pytest.raises(ValueError, match="Layout"):
        Graph("nope")
    with pytest.raises(ValueError, match="Strategy"):
        Graph("coco", "nope")


def test_sample_window_host():
    from temporal_inverse_kinematics_amd.windowing import InferenceDataset, sample_window
    w = golden("windowing.npz")
    for key in w.files:
        if not key.startswith("sw|"):
            continue
        parts = key.split("|")
        arr = w["arr20"][:10] if parts[1] == "10b" else (
            w["arr20"] if parts[1] == "20" else
            np.arange(10, dtype=np.float32)[:, None, None] * np.ones((1, 17, 3), np.float32))
        if parts[-1] == "err":
            with pytest.raises(ValueError):
                sample_window(arr, int(parts[2]), int(parts[3]))
        else:
            np.testing.assert_array_equal(sample_window(arr, int(parts[2]), int(parts[3])), w[key])
    ds = InferenceDataset(w["ids_in"], 9)
    items = np.stack([ds[i][0] for i in range(len(ds))])
    np.testing.assert_array_equal(items, w["ids_items"])


def test_keypoint_maps():
    from temporal_inverse_kinematics_amd import keypoints as kp
    k = golden("keypoints.npz")
    names = k["moveai_names"].tolist()
    assert kp.generate_moveai3d_to_coco_mappings(names) == list(k["moveai_to_coco"])
    assert kp.generate_smplx_to_coco_mappings(k["smplx_names"].tolist()) == list(k["smplx_to_coco"])
    np.testing.assert_array_equal(kp.moveai3d_to_coco(k["moveai_joints"], names), k["coco_seq"])


def test_synthetic_windows_shardable():
    from temporal_inverse_kinematics_amd import synthetic as syn
    full = syn.synthetic_windows(6, 16, seed=3)
    a = syn.synthetic_windows(3, 16, seed=3, start=0)
    b = syn.synthetic_windows(3, 16, seed=3, start=3)
    np.testing.assert_array_equal(np.concatenate([a, b]), full)
    root = 0.5 * (full[:, :, 11] + full[:, :, 12])
    assert np.abs(root).max() < 1e-6
    assert np.abs(full).max() < 2.5


def test_no_oracle_import_in_product():
    pkg = os.path.join(REPO, "temporal_inverse_kinematics_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(root, f)).read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", src).replace('"""', ""), f


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def test_bench_pmc_fields_only_from_this_tree(tmp_path, monkeypatch):
    """bench.py's roofline `traffic` / `mfma_busy` come only
    from a PMC summary measured on the benchmarked source tree (the summary
    carries _build.source_digest()); a summary of another tree gives null and
    says why, whatever its name."""
    import json
    from temporal_inverse_kinematics_amd._build import source_digest
    bench = _bench_module()
    sym = bench.kernel_symbol("XT128", "bf16x3")
    prof = tmp_path / "profiles"
    prof.mkdir()
    stale = {"source_digest": "0" * 16, "kernels": {sym: {"hbm_bytes_per_dispatch": 1.0}}}
    json.dump(stale, open(prof / "r99_z_pmc_traffic.json", "w"))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    v, src, note = bench._pmc_traffic(None, "XT128", "bf16x3")
    assert v is None and src is None and "this source tree" in note
    cur = {"source_digest": source_digest(), "kernels": {sym: {"hbm_bytes_per_dispatch": 7.0}}}
    json.dump(cur, open(prof / "r05_a_pmc_traffic.json", "w"))
    v, src, note = bench._pmc_traffic(None, "XT128", "bf16x3")
    assert v == 7.0 and src.endswith("r05_a_pmc_traffic.json")


def test_bench_kernel_symbols_resolve():
    """Every launch label of the default path maps to a symbol present in a
    committed rocprofv3 PMC summary (a templated kernel renamed in the
    profiler output once made the traffic field silently null)."""
    import glob
    import json
    bench = _bench_module()
    names = set()
    for p in glob.glob(os.path.join(REPO, "profiles", "*pmc_traffic*.json")):
        names |= {k.replace("void ", "").strip() for k in json.load(open(p)).get("kernels", {})}
    for label in ("XT128", "XH128", "XR", "XGW", "XTWG", "XB0", "XB1", "XG128", "XP64", "G0f_raw"):
        sym = bench.kernel_symbol(label, "bf16x3")
        assert sym and any(n == sym or ("<" not in sym and n.startswith(sym + "<")) for n in names), (label, sym)
