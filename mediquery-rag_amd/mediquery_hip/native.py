"""Thin handle classes over the C ABI: `FlatIndex` (mq_index_*) and `Encoder`
(mq_encoder_*).  Host calls take/return numpy arrays; `*_device` calls take torch
device tensors and run asynchronously on the given (or current) torch stream."""
import ctypes

import numpy as np

from . import _lib
from .config import BertConfig
from .weights import state_dict_to_blob, synthetic_state_dict


class FlatIndex:
    """HBM-resident exact cosine index (K8 add, K9 fused score + top-k, K10 merge)."""

    def __init__(self, dim=768, capacity=0, device=0, dtype=_lib.MQ_DTYPE_F32):
        h = ctypes.c_void_p()
        _lib.call("mq_index_create", device, dim, capacity, dtype, ctypes.byref(h))
        self._h = h
        self.dim = dim
        self.device = device

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            try:
                _lib.lib().mq_index_destroy(h)
            except Exception:  # interpreter shutdown
                pass

    __del__ = close

    def __len__(self):
        n = ctypes.c_int64()
        _lib.call("mq_index_size", self._h, ctypes.byref(n))
        return n.value

    def add(self, rows):
        rows = np.ascontiguousarray(rows, dtype=np.float32).reshape(-1, self.dim)
        _lib.call("mq_index_add", self._h, _lib.ptr(rows), rows.shape[0], 0, None)

    def add_device(self, rows, stream=None):
        assert rows.is_cuda and rows.dtype.is_floating_point and rows.is_contiguous()
        _lib.call("mq_index_add", self._h, _lib.ptr(rows), rows.shape[0], 1,
                  _lib.stream_handle(stream))

    def reset(self):
        _lib.call("mq_index_reset", self._h)

    def search(self, queries, k):
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dim)
        scores = np.empty((q.shape[0], k), dtype=np.float32)
        ids = np.empty((q.shape[0], k), dtype=np.int64)
        _lib.call("mq_index_search", self._h, _lib.ptr(q), q.shape[0], k, _lib.ptr(scores),
                  _lib.ptr(ids), 0, None)
        return scores, ids

    def search_device(self, queries, k, out_scores, out_ids, stream=None):
        """queries [nq, dim] f32, out_scores [nq, k] f32, out_ids [nq, k] int64 (torch, device)."""
        _lib.call("mq_index_search", self._h, _lib.ptr(queries), queries.shape[0], k,
                  _lib.ptr(out_scores), _lib.ptr(out_ids), 1, _lib.stream_handle(stream))

    def get(self, row0=0, n=None):
        """Stored (normalised) rows [row0, row0+n) as float32 numpy."""
        n = len(self) - row0 if n is None else n
        out = np.empty((n, self.dim), dtype=np.float32)
        _lib.call("mq_index_get", self._h, row0, n, _lib.ptr(out), 0, None)
        return out

    def select(self, rows, out=None):
        """Index whose row i is this index's row rows[i] (device gather, no host copy of
        the slab); out=self compacts in place.  Returns `out` (a new index if None)."""
        rows = np.ascontiguousarray(rows, dtype=np.int64).reshape(-1)
        out = FlatIndex(dim=self.dim, device=self.device) if out is None else out
        _lib.call("mq_index_select", self._h, _lib.ptr(rows), rows.size, out._h)
        return out

    def data_ptr(self):
        p = ctypes.c_void_p()
        _lib.call("mq_index_data", self._h, ctypes.byref(p))
        return p.value

    STAGES = ("flat_search_kernel", "merge_kernel")

    def set_precision(self, dtype):
        """_lib.MQ_DTYPE_F32 (exact f32 MFMA), _lib.MQ_DTYPE_F32X6 (split-f32),
        _lib.MQ_DTYPE_BF16 (bf16 coarse scan + exact fp32 re-rank) or
        _lib.MQ_DTYPE_F32_SCREEN (exact fp32 top-k: certified bf16 / split-f32 screens +
        fp32 re-rank)."""
        _lib.call("mq_index_set_precision", self._h, dtype)

    def set_stream_threshold(self, max_queries):
        """Batches of <= max_queries (0..16) use the streaming fp32 kernel (K9s)."""
        _lib.call("mq_index_set_stream_threshold", self._h, int(max_queries))

    def set_threshold_scan(self, enabled=True):
        """Batched bf16 candidate scans: threshold scan (K9t, default) or tiled lists."""
        _lib.call("mq_index_set_threshold_scan", self._h, int(bool(enabled)))

    def set_int8_screen(self, enabled=True):
        """Single screened queries: int8-shadow threshold scan first (K9q, default) or
        straight to the bf16 stream tier.  Same results either way."""
        _lib.call("mq_index_set_int8_screen", self._h, int(bool(enabled)))

    def set_async_screen(self, enabled=True):
        """Batched screened searches: uncertified queries re-run exactly on the device with
        no host read-back (default), or the synchronous tiered re-run.  Same results."""
        _lib.call("mq_index_set_async_screen", self._h, int(bool(enabled)))

    @property
    def rescans(self):
        """Searches whose k > 16 list-overflow check fired (re-scanned with 64 lists)."""
        n = ctypes.c_int64()
        _lib.call("mq_index_rescans", self._h, ctypes.byref(n), None)
        return n.value

    @property
    def remerges(self):
        """Merges whose 16-entry thread lists overflowed (re-run with 64)."""
        n = ctypes.c_int64()
        _lib.call("mq_index_rescans", self._h, None, ctypes.byref(n))
        return n.value

    @property
    def screen_fallbacks(self):
        """Screened queries (MQ_DTYPE_F32_SCREEN) re-run on the direct exact scan."""
        n = ctypes.c_int64()
        _lib.call("mq_index_screen_fallbacks", self._h, ctypes.byref(n), None)
        return n.value

    @property
    def screen_passdowns(self):
        """bf16-screened queries whose certificate failed, re-run on the split-f32 screen."""
        n = ctypes.c_int64()
        _lib.call("mq_index_screen_fallbacks", self._h, None, ctypes.byref(n))
        return n.value

    @property
    def screen_skips(self):
        """Batched screened searches that bypassed the bf16 tier (failure share > 0.2)."""
        n = ctypes.c_int64()
        _lib.call("mq_index_screen_skips", self._h, ctypes.byref(n), None)
        return n.value

    @property
    def int8_skips(self):
        """Single screened queries that sat the int8 tier out (failure share > 0.3)."""
        n = ctypes.c_int64()
        _lib.call("mq_index_screen_skips", self._h, None, ctypes.byref(n))
        return n.value

    def set_timing(self, enabled=True):
        _lib.call("mq_index_set_timing", self._h, int(bool(enabled)))

    def read_timing(self):
        """{stage: device ms since the last read} (HIP events on the launch stream)."""
        ms = np.zeros(len(self.STAGES), dtype=np.float32)
        _lib.call("mq_index_read_timing", self._h, _lib.ptr(ms), len(ms))
        return dict(zip(self.STAGES, ms.tolist()))

    def save(self, path):
        _lib.call("mq_index_save", self._h, str(path).encode())

    def load(self, path):
        _lib.call("mq_index_load", self._h, str(path).encode())

    def _check_bits(self, bits):
        check_mask_words(bits, len(self), self.device)

    def search_masked(self, queries, k, bits):
        """Exact top-k of each query ([dim] or [nq, dim] host floats) over the rows allowed
        by `bits` (a device mask tensor on this index's GPU of >= ceil(n / 32) int32 words,
        bit r % 32 of word r / 32 = row r; mask_eval builds it).  One call for the whole
        batch (mq_index_search_masked_batch).  -> (scores [nq, k], ids [nq, k])."""
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dim)
        self._check_bits(bits)
        scores = np.empty((q.shape[0], k), dtype=np.float32)
        ids = np.empty((q.shape[0], k), dtype=np.int64)
        with _lib.device_scope(self.device):
            _lib.call("mq_index_search_masked_batch", self._h, _lib.ptr(q), q.shape[0], k, _lib.ptr(bits),
                      _lib.ptr(scores), _lib.ptr(ids), 0, _lib.stream_handle(None))
        return scores, ids

    @property
    def masked_gathers(self):
        """Masked searches the int8 screen did not certify (answered from gathered rows)."""
        n = ctypes.c_int64()
        _lib.call("mq_index_masked_gathers", self._h, ctypes.byref(n))
        return n.value

    def save_rows(self, path, row0, n):
        """Rows [row0, row0 + n) as a slab file of n rows (a store segment)."""
        _lib.call("mq_index_save_rows", self._h, str(path).encode(), int(row0), int(n))

    def load_append(self, path):
        """Append a slab file's rows, bit-identical (no re-normalisation)."""
        _lib.call("mq_index_load_append", self._h, str(path).encode())


def merge_topk_host(scores, ids, k_out):
    """[n_lists, nq, k_in] candidate lists -> global top-k_out (score desc, id asc)."""
    scores = np.ascontiguousarray(scores, dtype=np.float32)
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    n_lists, nq, k_in = scores.shape
    os_ = np.empty((nq, k_out), dtype=np.float32)
    oi = np.empty((nq, k_out), dtype=np.int64)
    _lib.call("mq_topk_merge_host", _lib.ptr(scores), _lib.ptr(ids), n_lists, nq, k_in, k_out,
              _lib.ptr(os_), _lib.ptr(oi))
    return os_, oi


def merge_topk_device(scores, ids, k_out, out_scores, out_ids, stream=None):
    n_lists, nq, k_in = scores.shape
    _lib.call("mq_topk_merge_device", _lib.ptr(scores), _lib.ptr(ids), n_lists, nq, k_in, k_out,
              _lib.ptr(out_scores), _lib.ptr(out_ids), _lib.stream_handle(stream))


class Encoder:
    """BERT encoder on one GPU (K1..K7).  `weights`: HF-named state dict, or None for
    the seeded synthetic weights of `cfg` (see weights.py)."""

    def __init__(self, cfg: BertConfig, weights=None, seed=0, device=0):
        self.cfg = cfg
        self.device = device
        self._ccfg = _lib.BertConfigC.from_config(cfg)
        h = ctypes.c_void_p()
        _lib.call("mq_encoder_create", device, ctypes.byref(self._ccfg), ctypes.byref(h))
        self._h = h
        sd = weights if weights is not None else synthetic_state_dict(cfg, seed)
        blob = state_dict_to_blob(cfg, sd)
        n = _lib.lib().mq_encoder_weight_count(ctypes.byref(self._ccfg))
        if n != blob.size:
            raise ValueError("weight blob %d floats, library expects %d" % (blob.size, n))
        _lib.call("mq_encoder_load_weights", self._h, _lib.ptr(blob), blob.size)

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            try:
                _lib.lib().mq_encoder_destroy(h)
            except Exception:  # interpreter shutdown
                pass

    __del__ = close

    STAGES = ("embed_ln", "qkv_gemm", "attention", "out_proj_gemm", "layernorm", "ffn_up_gemm",
              "ffn_down_gemm", "pool")

    def set_timing(self, enabled=True):
        _lib.call("mq_encoder_set_timing", self._h, int(bool(enabled)))

    def read_timing(self):
        ms = np.zeros(len(self.STAGES), dtype=np.float32)
        _lib.call("mq_encoder_read_timing", self._h, _lib.ptr(ms), len(ms))
        return dict(zip(self.STAGES, ms.tolist()))

    def set_precision(self, dtype):
        _lib.call("mq_encoder_set_precision", self._h, dtype)

    def set_graphs(self, enabled=True):
        """Replay forwards as captured hipGraphs (default off: eager measured faster on
        MI355X for one query; bit-identical results)."""
        _lib.call("mq_encoder_set_graphs", self._h, int(bool(enabled)))

    OPTIONS = {"rows_max": _lib.MQ_ENC_OPT_ROWS_MAX, "rows_splits": _lib.MQ_ENC_OPT_ROWS_SPLITS,
               "splitk_max": _lib.MQ_ENC_OPT_SPLITK_MAX, "ln_rows_per_wave": _lib.MQ_ENC_OPT_LN_ROWS_PER_WAVE,
               "fuse_attn_oproj": _lib.MQ_ENC_OPT_FUSE_ATTN_OPROJ, "fused_ln": _lib.MQ_ENC_OPT_FUSED_LN,
               "splitk_tiles": _lib.MQ_ENC_OPT_SPLITK_TILES, "ln_on_load": _lib.MQ_ENC_OPT_LN_ON_LOAD,
               "resident_layers": _lib.MQ_ENC_OPT_RESIDENT_LAYERS, "x6_presplit": _lib.MQ_ENC_OPT_X6_PRESPLIT,
               "rows_planes": _lib.MQ_ENC_OPT_ROWS_PLANES}

    def set_option(self, name, value):
        """Tuning option of the forward (mq_encoder_set_option): rows_max, rows_splits,
        splitk_max, ln_rows_per_wave, fuse_attn_oproj, fused_ln, splitk_tiles, ln_on_load,
        resident_layers (0..1024, default 8: the few-row forward loads layers below this
        index with the default cache policy and later layers non-temporally, so the first
        layers' weights stay in MALL between single queries; outputs are bit-identical),
        x6_presplit (split-f32 precision: 1, default, multiplies the weights' W3 plane images
        split once at load; 0 = the tiles that re-split both operands; bit-identical),
        rows_planes (few-row forward: 0, default, merges the two-addend hand-offs into one plane
        by atomic adds; 1 = two planes; bit-identical)."""
        _lib.call("mq_encoder_set_option", self._h, self.OPTIONS[name], int(value))

    def get_option(self, name):
        v = ctypes.c_int()
        _lib.call("mq_encoder_get_option", self._h, self.OPTIONS[name], ctypes.byref(v))
        return v.value

    def embed(self, ids, mask):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        mask = np.ascontiguousarray(mask, dtype=np.int32)
        B, L = ids.shape
        out = np.empty((B, self.cfg.hidden), dtype=np.float32)
        _lib.call("mq_encoder_embed", self._h, _lib.ptr(ids), _lib.ptr(mask), B, L, _lib.ptr(out),
                  0, None)
        return out

    def embed_device(self, ids, mask, out, stream=None):
        """ids/mask int32 [B, L], out f32 [B, hidden] - torch device tensors."""
        B, L = ids.shape
        _lib.call("mq_encoder_embed", self._h, _lib.ptr(ids), _lib.ptr(mask), B, L, _lib.ptr(out),
                  1, _lib.stream_handle(stream))


def check_mask_words(bits, n, device=None):
    """A row mask for n rows: a contiguous 4-byte-element device tensor (on `device` when
    given) of >= ceil(n / 32) words - else ValueError (the kernels would read or write past
    its end, or on another GPU's memory)."""
    if not (getattr(bits, "is_cuda", False) and bits.element_size() == 4 and bits.is_contiguous()
            and bits.numel() >= (int(n) + 31) // 32):
        raise ValueError("bits must be a contiguous 32-bit device tensor of >= ceil(n / 32) = %d words"
                         % ((int(n) + 31) // 32))
    if device is not None and bits.device.index != int(device):
        raise ValueError("bits lives on cuda:%s, the index on cuda:%d" % (bits.device.index, int(device)))


def _check_codes(codes, bits):
    import torch
    if not (getattr(codes, "is_cuda", False) and codes.dtype == torch.int32 and codes.is_contiguous()):
        raise ValueError("codes must be a contiguous int32 device tensor")
    check_mask_words(bits, codes.numel(), codes.device.index)


def mask_eval(codes, lut, bits, mode, stream=None):
    """bits (mode)= lut[codes] on the device (include/mq.h mq_mask_eval): codes int32 [n]
    (-1 = key absent -> lut[-1]), lut uint8 [n_lut], bits int32 [ceil(n / 32)] (torch,
    one device; the launch runs there, on `stream` or that device's current stream)."""
    import torch
    _check_codes(codes, bits)
    if not (getattr(lut, "is_cuda", False) and lut.dtype == torch.uint8 and lut.is_contiguous()
            and lut.device == codes.device and lut.numel() >= 1):
        raise ValueError("lut must be a non-empty contiguous uint8 tensor on the codes' device")
    with _lib.device_scope(codes.device.index):
        _lib.call("mq_mask_eval", _lib.ptr(codes), codes.numel(), _lib.ptr(lut), lut.numel(), _lib.ptr(bits),
                  mode, _lib.stream_handle(stream))


def mask_eval_bits(codes, lut, bits, mode, stream=None):
    """mask_eval with a table of <= 256 entries passed by value (numpy bool / uint8 lut)."""
    _check_codes(codes, bits)
    lut = np.asarray(lut).astype(bool)
    if not 1 <= lut.size <= 256:
        raise ValueError("a by-value table holds 1..256 entries (got %d)" % lut.size)
    words = np.zeros(4, dtype=np.uint64)
    for i in np.flatnonzero(lut).tolist():
        words[i >> 6] |= np.uint64(1 << (i & 63))
    with _lib.device_scope(codes.device.index):
        _lib.call("mq_mask_eval_bits", _lib.ptr(codes), codes.numel(), _lib.ptr(words), len(lut), _lib.ptr(bits),
                  mode, _lib.stream_handle(stream))


def mask_combine(dst, src, mode, stream=None):
    """dst (mode)= src (None: all ones; MQ_MASK_CLEAR: zeros) on the device."""
    check_mask_words(dst, 0)
    if src is not None:
        check_mask_words(src, 32 * dst.numel(), dst.device.index)
    with _lib.device_scope(dst.device.index):
        _lib.call("mq_mask_combine", _lib.ptr(dst), _lib.ptr(src), dst.numel(), mode, _lib.stream_handle(stream))

