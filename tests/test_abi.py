"""The C-ABI library loads here (no GPU), exports every symbol include/mq.h declares,
and its pure-host entry points behave; device entry points fail loudly without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

from mediquery_hip import _lib
from mediquery_hip.config import BertConfig, DMETA_BASE
from mediquery_hip.native import merge_topk_host
from mediquery_hip.weights import blob_size, hf_names, state_dict_to_blob, synthetic_state_dict

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "mq.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(mq_\w+)\s*\(", text, re.M)))


def test_header_symbols_exported_and_bound():
    syms = declared_symbols()
    assert len(syms) >= 20
    h = _lib.lib()
    for s in syms:
        assert hasattr(h, s), s
        assert s in _lib.SIGNATURES, "no ctypes signature for " + s


def test_version_and_device_count():
    assert b"gfx950" in _lib.lib().mq_version()
    assert _lib.device_count() >= 0


def test_library_built_from_this_tree():
    """The .so carries the hash of the sources it was compiled from (csrc/Makefile
    STAMPED); it equals the tree's, so the library the GPU runs is not a stale prebuilt."""
    built = _lib.built_source_hash()
    assert len(built) == 16 and int(built, 16) >= 0
    assert built == _lib.tree_source_hash()
    _lib.check_build_fresh()


def test_weight_count_matches_python_layout():
    for cfg in (DMETA_BASE, BertConfig(layers=2)):
        c = _lib.BertConfigC.from_config(cfg)
        assert _lib.lib().mq_encoder_weight_count(ctypes.byref(c)) == blob_size(cfg)


def test_blob_layout_roundtrip():
    cfg = BertConfig(vocab_size=300, hidden=256, layers=2, heads=4, ffn=512, max_positions=64)
    sd = synthetic_state_dict(cfg, 3)
    blob = state_dict_to_blob(cfg, sd)
    assert blob.size == blob_size(cfg)
    H = cfg.hidden
    off = (300 + 64 + 2) * H + 2 * H
    wq = sd["encoder.layer.0.attention.self.query.weight"]
    wk = sd["encoder.layer.0.attention.self.key.weight"]
    np.testing.assert_array_equal(blob[off:off + H * H].reshape(H, H), wq)
    np.testing.assert_array_equal(blob[off + H * H:off + 2 * H * H].reshape(H, H), wk)
    assert len(hf_names(cfg)) == 5 + 16 * cfg.layers


def _merge_ref(s, i, k):
    n_lists, nq, kin = s.shape
    out_i = []
    for q in range(nq):
        pool = [(-s[l, q, j], i[l, q, j]) for l in range(n_lists) for j in range(kin) if i[l, q, j] >= 0]
        pool.sort()
        out_i.append([p[1] for p in pool[:k]] + [-1] * max(0, k - len(pool)))
    return np.array(out_i)


def test_host_merge_matches_sort():
    r = np.random.default_rng(0)
    s = np.round(r.random((6, 9, 5)), 2).astype(np.float32)  # rounding forces score ties
    i = r.permutation(6 * 9 * 5).reshape(6, 9, 5).astype(np.int64)
    i[0, 0, :] = -1                                            # padding entries
    os_, oi = merge_topk_host(s, i, 7)
    np.testing.assert_array_equal(oi, _merge_ref(s, i, 7))
    assert np.all(np.diff(os_, axis=1) <= 0)


def test_host_merge_pads_when_short():
    s = np.array([[[0.5, -np.inf]]], np.float32)
    i = np.array([[[3, -1]]], np.int64)
    os_, oi = merge_topk_host(s, i, 3)
    assert oi.tolist() == [[3, -1, -1]] and np.isneginf(os_[0, 1:]).all()


def test_bad_arguments_raise_with_message():
    h = ctypes.c_void_p()
    with pytest.raises(_lib.MQError, match="dim must be"):
        _lib.call("mq_index_create", 0, 100, 0, 0, ctypes.byref(h))
    with pytest.raises(_lib.MQError, match="bad merge shape"):
        _lib.call("mq_topk_merge_host", None, None, 0, 1, 1, 1, None, None)
